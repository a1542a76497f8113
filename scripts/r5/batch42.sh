#!/bin/bash
# r5 batch 42: forward consumer-side BN apply (conv2 -> conv3 prologue): tests + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_fwd_pro.py tests/test_gpu_bnfold.py \
  tests/test_gpu_resnet50_parity.py tests/test_gpu_pw.py > gpurun_out/r5/b42_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b42_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b42_pro_$i.log 2>&1 || exit 10
  ZOO_FWD_PRO=0 $T 200 python -u bench.py > gpurun_out/r5/b42_apply_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b42_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
