#!/bin/bash
# r5 batch 44: igemm2 for the 128-wide stage-2 3x3 convs per direction (forward / dgrad)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
ZOO_I2_KMIN_FWD=128 ZOO_I2_KMIN_BWD=128 $T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_resnet50_parity.py > gpurun_out/r5/b44_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b44_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b44_def_$i.log 2>&1 || exit 10
  ZOO_I2_KMIN_FWD=128 $T 200 python -u bench.py > gpurun_out/r5/b44_fwd128_$i.log 2>&1 || exit 11
  ZOO_I2_KMIN_BWD=128 $T 200 python -u bench.py > gpurun_out/r5/b44_bwd128_$i.log 2>&1 || exit 12
done
for f in gpurun_out/r5/b44_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
