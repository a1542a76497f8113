#!/bin/bash
# r5 round-end check: full GPU test suite, smoke(), default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5/final_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5/final_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
$T 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/final_smoke.log 2>&1 || exit 20
tail -1 gpurun_out/r5/final_smoke.log
$T 200 python -u bench.py > gpurun_out/r5/final_bench.log 2>&1 || exit 21
tail -1 gpurun_out/r5/final_bench.log
