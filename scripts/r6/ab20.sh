#!/bin/bash
# r6 run 20: persistent row-group ConvLSTM step kernel -- tests, then fused vs fused_np vs loop (3-D 32^3 T = 16)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "convlstm or ConvLSTM" > gpurun_out/r6/ab20_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab20_tests.log; [ $rc -ne 0 ] && exit $rc
$T 300 python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes loop,fused,fused_np --iters 5 > gpurun_out/r6/ab20_cl3d.log 2>&1 || exit 42
$T 300 python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes fused,fused_np --iters 5 >> gpurun_out/r6/ab20_cl3d.log 2>&1 || exit 43
grep bench gpurun_out/r6/ab20_cl3d.log
