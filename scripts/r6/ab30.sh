#!/bin/bash
# r6 run 30: ResNet-50 featureset bench step -- full names of the PyTorch / runtime dispatches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
rm -rf /tmp/prof_rn30
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_rn30 -o rn -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/r6/ab30_bench.log 2>&1 || exit 44
DB=$(find /tmp/prof_rn30 -name "*.db" | head -1)
python3 scripts/r6/step_small.py $DB > gpurun_out/r6/ab30_small.txt 2>&1
cut -c1-330 gpurun_out/r6/ab30_small.txt
