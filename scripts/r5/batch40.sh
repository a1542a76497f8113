#!/bin/bash
# r5 batch 40: 64-row tiles of the tiled weight gradient (K <= 64 convs, incl. the stem) vs 128-row + DMA
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b40_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_BM64=0 $T 200 python -u bench.py > gpurun_out/r5/b40_bm128_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b40_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
