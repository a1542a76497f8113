#!/bin/bash
# r6 run 7: ConvLSTM3D per-kernel totals (fused vs per-step loop), then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
for mode in fused loop; do
  rm -rf /tmp/prof_cl_$mode
  $T 300 rocprofv3 --kernel-trace -d /tmp/prof_cl_$mode -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes $mode --iters 3 > gpurun_out/r6/ab7_cl_$mode.log 2>&1 || exit 41
  DB=$(find /tmp/prof_cl_$mode -name "*.db" | head -1)
  python3 analytics-zoo_amd/tools/prof_step.py $DB --totals > gpurun_out/r6/ab7_cl_${mode}_totals.md 2>&1
  head -24 gpurun_out/r6/ab7_cl_${mode}_totals.md | cut -c1-200
done
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab7_gpu_suite.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab7_gpu_suite.log; exit $rc
