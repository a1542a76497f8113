#!/bin/bash
# r5 batch 13: CU-masked weight-gradient side stream A/B (ZOO_SIDE_CUS), ConvLSTM with LDS weights
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_convlstm_seq.py \
  tests/test_gpu_keras_native.py -k "ConvLSTM or convlstm" > gpurun_out/r5/b13_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b13_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b13_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b13_convlstm_bench.log
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b13_cu0_$i.log 2>&1 || exit 10
  ZOO_SIDE_CUS=32 $T 200 python -u bench.py > gpurun_out/r5/b13_cu32_$i.log 2>&1 || exit 11
  ZOO_SIDE_CUS=64 $T 200 python -u bench.py > gpurun_out/r5/b13_cu64_$i.log 2>&1 || exit 12
  ZOO_SIDE_CUS=16 $T 200 python -u bench.py > gpurun_out/r5/b13_cu16_$i.log 2>&1 || exit 13
done
for f in gpurun_out/r5/b13_cu*_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
$T 600 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/b13_quant.log 2>&1 || exit 7
tail -1 gpurun_out/r5/b13_quant.log | head -c 3000
