#!/bin/bash
# r6 run 10: single-GEMM conv3d (depth taps on channels): Conv3D / ConvLSTM3D tests and bench, then
# the whole GPU suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab10_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab10_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in "--dims 3 --T 16" "--dims 3 --T 16 --hw 16"; do
  $T 300 python3 -u analytics-zoo_amd/tools/convlstm_bench.py $cfg >> gpurun_out/r6/ab10_convlstm.log 2>&1 || exit 41
done
grep '"bench"' gpurun_out/r6/ab10_convlstm.log | cut -c1-200
$T 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab10_gpu_suite.log 2>&1
rc=$?; tail -6 gpurun_out/r6/ab10_gpu_suite.log; exit $rc
