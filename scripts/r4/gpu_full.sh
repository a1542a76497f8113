#!/bin/bash
# Full GPU test suite + smoke + default bench (the driver's round-end sequence), one call
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 5
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 200 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 6
tail -1 gpurun_out/bench_$TAG.log
