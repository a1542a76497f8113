#!/bin/bash
# r5 batch 56: HBM bytes per kernel family of the ResNet-50 step (PMC: FETCH_SIZE, WRITE_SIZE in separate passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pmc_fetch -o f -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/r5/b56_fetch.log" 2>&1 || exit 10
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pmc_write -o w -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/r5/b56_write.log" 2>&1 || exit 11
cd "$GRAFT_REPO_ROOT"
python3 analytics-zoo_amd/tools/pmc_summary.py $(find /tmp/pmc_fetch -name "*.db" | head -1) > gpurun_out/r5/b56_fetch_summary.txt 2>&1
python3 analytics-zoo_amd/tools/pmc_summary.py $(find /tmp/pmc_write -name "*.db" | head -1) > gpurun_out/r5/b56_write_summary.txt 2>&1
head -40 gpurun_out/r5/b56_fetch_summary.txt
