#!/bin/bash
# r5 batch 65: ResNet-50 with / without the in-backward optimizer
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b65_def_$i.log 2>&1 || exit 10
  ZOO_OPTIM_IN_BWD=0 $T 200 python -u bench.py > gpurun_out/r5/b65_noibo_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b65_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
