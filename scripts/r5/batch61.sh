#!/bin/bash
# r5 batch 61: MobileNet-v1 b64 training, wgrad knob A/B with repetitions
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
B="python -u analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 60"
for i in 1 2 3; do
  $T 300 $B > gpurun_out/r5/b61_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_WG=1024 $T 300 $B > gpurun_out/r5/b61_wg1024_$i.log 2>&1 || exit 11
  ZOO_WGRAD_DMA=0 $T 300 $B > gpurun_out/r5/b61_nodma_$i.log 2>&1 || exit 12
done
for f in gpurun_out/r5/b61_*_?.log; do echo "$f $(grep -o '"img_s": [0-9.]*' $f)"; done
