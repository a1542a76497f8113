#!/bin/bash
# r6 run 9: ConvLSTM step kernels with two pixel blocks per wave (tests + 3-D / 2-D bench), ResNet-50
# same-box A/B of the transposed band weight gradient on the default (featureset) bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py -k "convlstm or ConvLSTM" \
  -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab9_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab9_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in "--dims 3 --T 16" "--dims 3 --T 16 --hw 16" "--dims 2 --T 16" "--dims 2 --T 32"; do
  $T 300 python3 -u analytics-zoo_amd/tools/convlstm_bench.py $cfg >> gpurun_out/r6/ab9_convlstm.log 2>&1 || exit 41
done
grep '"bench"' gpurun_out/r6/ab9_convlstm.log | cut -c1-260
for i in 1 2 3; do
  for b in 2 1; do
    ZOO_WGRAD_BAND=$b $T 300 python -u bench.py > gpurun_out/r6/ab9_fs_band${b}_$i.log 2>&1 || exit 22
    echo "band$b $(tail -1 gpurun_out/r6/ab9_fs_band${b}_$i.log | cut -c60-120)"
  done
done
