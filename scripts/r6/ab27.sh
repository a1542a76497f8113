#!/bin/bash
# r6 run 27: one ConvLSTM3D fused iteration's dispatch timeline (32^3, T = 16)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
rm -rf /tmp/prof_cl27
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_cl27 -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes fused --iters 2 > gpurun_out/r6/ab27_cl_fused.log 2>&1 || exit 44
DB=$(find /tmp/prof_cl27 -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB "igemm_kernel<8, false, false, 64, true, 1>" 1 > gpurun_out/r6/ab27_cl_step.md 2>&1
grep -v "pers_kernel" gpurun_out/r6/ab27_cl_step.md | cut -c1-170
