#!/bin/bash
# r5 batch 36: re-sweep of the BN pass grid and the weight-gradient split floor on the new defaults
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b36_def_$i.log 2>&1 || exit 10
  ZOO_BN_BLOCKS=512 $T 200 python -u bench.py > gpurun_out/r5/b36_bnb512_$i.log 2>&1 || exit 11
  ZOO_BN_BLOCKS=2048 $T 200 python -u bench.py > gpurun_out/r5/b36_bnb2048_$i.log 2>&1 || exit 12
  ZOO_WGRAD_MINPIX=1024 $T 200 python -u bench.py > gpurun_out/r5/b36_mp1024_$i.log 2>&1 || exit 13
  ZOO_WGRAD256_ATOMIC_MB=64 $T 200 python -u bench.py > gpurun_out/r5/b36_amb64_$i.log 2>&1 || exit 14
done
for f in gpurun_out/r5/b36_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
