#!/bin/bash
# r5 batch 33: weight-gradient workgroup target sweep (+ DMA staging)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  ZOO_WGRAD_WG=512 $T 200 python -u bench.py > gpurun_out/r5/b33_wg512_$i.log 2>&1 || exit 10
  ZOO_WGRAD_WG=256 $T 200 python -u bench.py > gpurun_out/r5/b33_wg256_$i.log 2>&1 || exit 11
  ZOO_WGRAD_WG=384 $T 200 python -u bench.py > gpurun_out/r5/b33_wg384_$i.log 2>&1 || exit 12
  ZOO_WGRAD_WG=512 ZOO_WGRAD_DMA=1 $T 200 python -u bench.py > gpurun_out/r5/b33_wg512dma_$i.log 2>&1 || exit 13
  ZOO_WGRAD_WG=256 ZOO_WGRAD_DMA=1 $T 200 python -u bench.py > gpurun_out/r5/b33_wg256dma_$i.log 2>&1 || exit 14
done
for f in gpurun_out/r5/b33_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
