#!/bin/bash
# round-3 final check: full GPU suite, smoke, default bench (driver contract)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r3final_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3final_full.log; [ $rc = 0 ] || exit 1
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 2
tail -1 gpurun_out/smoke_final.log
$T 300 python -u bench.py > gpurun_out/bench_final_default.log 2>&1 || exit 3
tail -1 gpurun_out/bench_final_default.log
echo done
