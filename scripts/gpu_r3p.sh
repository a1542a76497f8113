#!/bin/bash
# round-3 batch P: ResNet-50 kernel profile after the implicit wgrad256, per-shape conv sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u analytics-zoo_amd/tools/conv_sweep.py --detail > gpurun_out/conv_sweep_p.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/conv_sweep_p.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_rn_p.log 2>&1 || exit 2
cd $GRAFT_REPO_ROOT
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_rn -name "*.db" | head -1) 8 "ResNet-50 b256 training (bench.py --steps 5 --warmup 3 under rocprofv3; 8 steps traced)" > gpurun_out/prof_rn_p_summary.md 2>&1
head -40 gpurun_out/prof_rn_p_summary.md
echo done
