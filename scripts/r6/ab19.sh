#!/bin/bash
# r6 run 19: ConvLSTM3D fused per-kernel totals on the current code (32^3, T = 16)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
rm -rf /tmp/prof_cl_fused
$T 300 rocprofv3 --kernel-trace -d /tmp/prof_cl_fused -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes fused --iters 3 > gpurun_out/r6/ab19_cl_fused.log 2>&1 || exit 41
DB=$(find /tmp/prof_cl_fused -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --totals > gpurun_out/r6/ab19_cl_fused_totals.md 2>&1
head -30 gpurun_out/r6/ab19_cl_fused_totals.md | cut -c1-200
