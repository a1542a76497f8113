#!/bin/bash
# r5 batch 17: ConvLSTM step kernels in isolation (kernel trace + one counter pass)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
$T 2>/dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cs -o cs -- python3 analytics-zoo_amd/tools/convlstm_step_bench.py > gpurun_out/r5/b17_cs.log 2>&1 || exit 2
DB=$(find /tmp/prof_cs -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM step kernels" > gpurun_out/r5/b17_cs_summary.md 2>&1
grep -E "convlstm" gpurun_out/r5/b17_cs_summary.md
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_MFMA -d /tmp/prof_cs2 -o cs2 -- python3 analytics-zoo_amd/tools/convlstm_step_bench.py --iters 2 > gpurun_out/r5/b17_pmc.log 2>&1 || exit 3
find /tmp/prof_cs2 -name "*counter_collection.csv" -exec cp {} gpurun_out/r5/b17_pmc.csv \;
ls -la gpurun_out/r5/b17_pmc.csv
