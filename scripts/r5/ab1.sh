#!/bin/bash
# r5 A/B 1: high-priority compute stream; compute-stream-alone profile (side stream off); IBO tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_ibo.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5/ibo_tests.log 2>&1 || { tail -30 gpurun_out/r5/ibo_tests.log; exit 3; }
tail -3 gpurun_out/r5/ibo_tests.log
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/ab1_def_$i.log 2>&1 || exit 4
  ZOO_COMPUTE_PRIORITY=1 $T 200 python -u bench.py > gpurun_out/r5/ab1_prio_$i.log 2>&1 || exit 5
done
grep -h '"metric"' gpurun_out/r5/ab1_*.log | cut -c1-200
ZOO_WGRAD_STREAM=0 $T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ws0 -o ws0 -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/r5/prof_ws0.log 2>&1 || exit 8
DB=$(find /tmp/prof_ws0 -name "*.db" | head -1)
cp $DB gpurun_out/r5/ws0.db
python3 analytics-zoo_amd/tools/prof_summary.py $DB 11 "ResNet-50 b256, weight-gradient side stream OFF (compute alone)" > gpurun_out/r5/prof_ws0_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r5/prof_ws0_step.md 2>&1
tail -8 gpurun_out/r5/prof_ws0_step.md
