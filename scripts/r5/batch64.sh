#!/bin/bash
# r5 batch 64: NCF with / without the in-backward optimizer
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 300 python -u bench.py --model ncf --batch 65536 --steps 100 --warmup 20 > gpurun_out/r5/b64_def_$i.log 2>&1 || exit 10
  ZOO_OPTIM_IN_BWD=0 $T 300 python -u bench.py --model ncf --batch 65536 --steps 100 --warmup 20 > gpurun_out/r5/b64_noibo_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b64_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
