#!/bin/bash
# r5 batch 60: MobileNet-v1 b64 training vs the round-5 wgrad defaults (512 WG, DMA) -- regression check
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 300 python -u analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 40 > gpurun_out/r5/b60_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_WG=1024 ZOO_WGRAD_DMA=0 $T 300 python -u analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 40 > gpurun_out/r5/b60_r4_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b60_*_?.log; do echo "$f $(grep -o '"img_s": [0-9.]*' $f)"; done
