#!/bin/bash
# persistent-kernel contention A/B: c3 band-run split and pw oversubscription (dispatcher-balanced)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b6_def_$i.log 2>&1 || exit 10
  ZOO_C3_SPLIT=2 $T 200 python -u bench.py > gpurun_out/r5/b6_c3s2_$i.log 2>&1 || exit 11
  ZOO_C3_SPLIT=4 $T 200 python -u bench.py > gpurun_out/r5/b6_c3s4_$i.log 2>&1 || exit 12
  ZOO_PW_OVERSUB=2 $T 200 python -u bench.py > gpurun_out/r5/b6_pw2_$i.log 2>&1 || exit 13
  ZOO_PW_OVERSUB=4 $T 200 python -u bench.py > gpurun_out/r5/b6_pw4_$i.log 2>&1 || exit 14
done
for f in gpurun_out/r5/b6_{def,c3s2,c3s4,pw2,pw4}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
