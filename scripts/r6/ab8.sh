#!/bin/bash
# r6 run 8: residual-prologue fallback + s2d 32-bit index tests, qconv suite, ResNet benches,
# input-pass kernel times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_fwd_pro.py tests/test_gpu_qconv.py tests/test_gpu_kernels.py -k "pro or qconv or int8 or fp8 or s2d" \
  -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab8_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab8_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  $T 300 python -u bench.py > gpurun_out/r6/ab8_fs_$i.log 2>&1 || exit 22
  tail -1 gpurun_out/r6/ab8_fs_$i.log | cut -c1-160
  $T 300 python -u bench.py --input device > gpurun_out/r6/ab8_dev_$i.log 2>&1 || exit 22
  tail -1 gpurun_out/r6/ab8_dev_$i.log | cut -c1-160
done
rm -rf /tmp/prof_fs
$T 300 rocprofv3 --kernel-trace -d /tmp/prof_fs -o fs -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/r6/ab8_prof_fs.log 2>&1 || exit 8
DB=$(find /tmp/prof_fs -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --totals > gpurun_out/r6/ab8_prof_fs_totals.md 2>&1
grep -E "s2d|maxpool|total kernel" gpurun_out/r6/ab8_prof_fs_totals.md | cut -c1-160
