#!/bin/bash
# rocprofv3 kernel trace of the ResNet-50 b256 bench step: per-kernel summary + one-step timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
TAG=${1:-r4}
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/prof_rn_$TAG.log 2>&1 || exit 8
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 11 "ResNet-50 b256 training (bench.py under rocprofv3), $TAG" > gpurun_out/prof_rn_${TAG}_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB > gpurun_out/prof_rn_${TAG}_step.md 2>&1
head -40 gpurun_out/prof_rn_${TAG}_summary.md
