#!/bin/bash
# r5 batch 19: BN-backward prologue at K = 128 (64-channel groups): tests + same-box A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
ZOO_BN_FOLD_K=64,128 $T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfold.py > gpurun_out/r5/b19_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b19_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b19_k64_$i.log 2>&1 || exit 10
  ZOO_BN_FOLD_K=64,128 $T 200 python -u bench.py > gpurun_out/r5/b19_k128_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b19_{k64,k128}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
