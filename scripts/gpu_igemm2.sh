#!/bin/bash
# igemm2 numerics tests then the kernel A/B bench; stops on anything worse than a test failure
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_igemm2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_igemm2.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t_igemm2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u analytics-zoo_amd/tools/igemm2_bench.py ${BENCH_ARGS} --out gpurun_out/igemm2_bench.json > gpurun_out/igemm2_bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -3 gpurun_out/igemm2_bench.log
exit $rc2
