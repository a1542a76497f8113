#!/bin/bash
# r5 A/B 2: split-K weight-gradient reduction by fp32 atomics (wgrad256 ZOO_WGRAD256_ATOMIC_MB;
# wgrad.hip ZOO_WGRAD_PARTIAL_MB) vs partials + fold kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_wgrad256.py tests/test_gpu_resnet50_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5/ab2_tests.log 2>&1 || { tail -30 gpurun_out/r5/ab2_tests.log; exit 3; }
tail -2 gpurun_out/r5/ab2_tests.log
for i in 1 2; do
  ZOO_WGRAD256_ATOMIC_MB=0 $T 200 python -u bench.py > gpurun_out/r5/ab2_off_$i.log 2>&1 || exit 4
  $T 200 python -u bench.py > gpurun_out/r5/ab2_def_$i.log 2>&1 || exit 5
  ZOO_WGRAD256_ATOMIC_MB=100000 ZOO_WGRAD_PARTIAL_MB=0 $T 200 python -u bench.py > gpurun_out/r5/ab2_all_$i.log 2>&1 || exit 6
done
for f in gpurun_out/r5/ab2_{off,def,all}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab2 -o ab2 -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/r5/prof_ab2.log 2>&1 || exit 8
DB=$(find /tmp/prof_ab2 -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 11 "ResNet-50 b256, atomic split-K wgrad (default)" > gpurun_out/r5/prof_ab2_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r5/prof_ab2_step.md 2>&1
tail -3 gpurun_out/r5/prof_ab2_step.md
