#!/bin/bash
# r5 batch 39: weight-gradient routing of the 64-channel stage-1 convs (CMIN / CONV_COUT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b39_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD256_CMIN=64 $T 200 python -u bench.py > gpurun_out/r5/b39_cmin64_$i.log 2>&1 || exit 11
  ZOO_WGRAD256_CONV_COUT=512 $T 200 python -u bench.py > gpurun_out/r5/b39_cout512_$i.log 2>&1 || exit 12
  ZOO_WGRAD256_CMIN=64 ZOO_WGRAD256_CONV_COUT=512 $T 200 python -u bench.py > gpurun_out/r5/b39_both_$i.log 2>&1 || exit 13
done
for f in gpurun_out/r5/b39_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
