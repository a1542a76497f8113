#!/bin/bash
# r6 run 36: round-end validation -- full GPU suite (skips named), smoke(), default bench x2, ConvLSTM3D bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab36_gpu_suite.log 2>&1
rc=$?; tail -6 gpurun_out/r6/ab36_gpu_suite.log; [ $rc -ne 0 ] && exit $rc
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/ab36_smoke.log 2>&1 || exit 45
tail -2 gpurun_out/r6/ab36_smoke.log
for i in 1 2; do
  $T 400 python -u bench.py > gpurun_out/r6/ab36_bench_$i.log 2>&1 || exit 46
  grep '"metric"' gpurun_out/r6/ab36_bench_$i.log | cut -c1-200
done
for cfg in "--dims 3 --T 16" "--dims 3 --T 16 --hw 16" "--dims 2 --T 16"; do
  $T 300 python3 -u analytics-zoo_amd/tools/convlstm_bench.py $cfg --iters 5 >> gpurun_out/r6/ab36_convlstm.log 2>&1 || exit 47
done
grep '"bench"' gpurun_out/r6/ab36_convlstm.log | cut -c1-220
