#!/bin/bash
# r5 batch 18: ConvLSTM step kernels with the epilogue operands prefetched before the GEMM
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_convlstm_seq.py \
  tests/test_gpu_keras_native.py -k "ConvLSTM or convlstm" > gpurun_out/r5/b18_cl_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b18_cl_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b18_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b18_convlstm_bench.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cs -o cs -- python3 analytics-zoo_amd/tools/convlstm_step_bench.py > gpurun_out/r5/b18_cs.log 2>&1 || exit 2
DB=$(find /tmp/prof_cs -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM step kernels" > gpurun_out/r5/b18_cs_summary.md 2>&1
grep -E "convlstm" gpurun_out/r5/b18_cs_summary.md
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cl -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --iters 3 > gpurun_out/r5/b18_prof_cl.log 2>&1 || exit 12
DB=$(find /tmp/prof_cl -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM2D T=32 bench (3 modes)" > gpurun_out/r5/b18_prof_cl_summary.md 2>&1
head -30 gpurun_out/r5/b18_prof_cl_summary.md
