#!/bin/bash
# r5 batch 7: full GPU suite (the driver's round-end tier) + smoke; quant clip sweep + per-block diag
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5/pytest_gpu_full_b7.log 2>&1
rc=$?
tail -15 gpurun_out/r5/pytest_gpu_full_b7.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/smoke_b7.log 2>&1 || exit 5
tail -2 gpurun_out/r5/smoke_b7.log
$T 300 python -u analytics-zoo_amd/tools/quant_diag.py > gpurun_out/r5/quant_diag_ch.log 2>&1 || exit 6
tail -1 gpurun_out/r5/quant_diag_ch.log
$T 600 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/quant_bench_b7.log 2>&1 || exit 7
tail -1 gpurun_out/r5/quant_bench_b7.log
