#!/bin/bash
# r6 run 28: ConvLSTM3D fused path on the bf16 gate input / gradient -- tests, A/B, per-kernel totals
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "convlstm or ConvLSTM or onv3D or conv3d or onvolution3D or Pooling3D" > gpurun_out/r6/ab28_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab28_tests.log; [ $rc -ne 0 ] && exit $rc
$T 300 python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes loop,fused,fused_rg,fused_np --iters 5 > gpurun_out/r6/ab28_cl3d.log 2>&1 || exit 42
$T 300 python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --hw 16 --modes loop,fused --iters 5 >> gpurun_out/r6/ab28_cl3d.log 2>&1 || exit 43
grep bench gpurun_out/r6/ab28_cl3d.log
rm -rf /tmp/prof_cl_fused
$T 300 rocprofv3 --kernel-trace -d /tmp/prof_cl_fused -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes fused --iters 3 > gpurun_out/r6/ab28_cl_fused.log 2>&1 || exit 44
DB=$(find /tmp/prof_cl_fused -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --totals > gpurun_out/r6/ab28_cl_fused_totals.md 2>&1
head -24 gpurun_out/r6/ab28_cl_fused_totals.md | cut -c1-160
