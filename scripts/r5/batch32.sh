#!/bin/bash
# r5 batch 32: weight-gradient split / staging knobs A/B on the ResNet-50 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b32_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_WG=512 $T 200 python -u bench.py > gpurun_out/r5/b32_wg512_$i.log 2>&1 || exit 11
  ZOO_WGRAD_WG=2048 $T 200 python -u bench.py > gpurun_out/r5/b32_wg2048_$i.log 2>&1 || exit 12
  ZOO_WGRAD_DMA=1 $T 200 python -u bench.py > gpurun_out/r5/b32_dma_$i.log 2>&1 || exit 13
done
for f in gpurun_out/r5/b32_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
