#!/bin/bash
# round-3 batch N: full GPU suite, smoke, bench (round-end rehearsal)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_full_n.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/t_full_n.log; [ $rc = 0 ] || exit 1
$T 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_n.log 2>&1 || { tail -20 gpurun_out/smoke_n.log; exit 2; }
tail -1 gpurun_out/smoke_n.log
$T 300 python -u bench.py > gpurun_out/bench_n.log 2>&1 || { tail -20 gpurun_out/bench_n.log; exit 3; }
grep '"metric"' gpurun_out/bench_n.log
echo done
