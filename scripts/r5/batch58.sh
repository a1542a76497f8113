#!/bin/bash
# r5 batch 58: stem max-pool forward with two outputs per thread (15 loads for 2 windows): tests + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_stem_pool.py tests/test_gpu_resnet50_parity.py \
  > gpurun_out/r5/b58_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b58_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b58_fwd2_$i.log 2>&1 || exit 10
  ZOO_POOL_FWD2=0 $T 200 python -u bench.py > gpurun_out/r5/b58_fwd1_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b58_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
