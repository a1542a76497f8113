#!/bin/bash
# r5 batch 43: forward consumer-side apply restricted to the 64-channel units
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  ZOO_FWD_PRO_K=64 $T 200 python -u bench.py > gpurun_out/r5/b43_k64_$i.log 2>&1 || exit 10
  ZOO_FWD_PRO=0 $T 200 python -u bench.py > gpurun_out/r5/b43_apply_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b43_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
