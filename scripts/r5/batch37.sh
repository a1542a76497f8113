#!/bin/bash
# r5 batch 37: stage-1 1x1 weight gradients back on the tiled kernel (new 512-WG / DMA defaults)?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b37_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD256_MMAX=262144 $T 200 python -u bench.py > gpurun_out/r5/b37_mmax18_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b37_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
