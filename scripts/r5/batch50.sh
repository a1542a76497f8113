#!/bin/bash
# r5 batch 50: BN-backward prologue at K = 128 / 256 with single-buffered y fragments (no spills)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
ZOO_BN_FOLD_K=64,128,256 $T 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bnfold.py \
  tests/test_gpu_resnet50_parity.py tests/test_gpu_pw.py > gpurun_out/r5/b50_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b50_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b50_k64_$i.log 2>&1 || exit 10
  ZOO_BN_FOLD_K=64,256 $T 200 python -u bench.py > gpurun_out/r5/b50_k256_$i.log 2>&1 || exit 11
  ZOO_BN_FOLD_K=64,128,256 $T 200 python -u bench.py > gpurun_out/r5/b50_kall_$i.log 2>&1 || exit 12
  ZOO_BN_FOLD_K=64,128 $T 200 python -u bench.py > gpurun_out/r5/b50_k128_$i.log 2>&1 || exit 13
done
for f in gpurun_out/r5/b50_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
