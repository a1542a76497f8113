set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_zoo_kernels.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pool.log 2>&1 || exit 1
$T 200 python bench.py > gpurun_out/bench_pool1.log 2>&1 || exit 2
$T 200 python bench.py > gpurun_out/bench_pool2.log 2>&1 || exit 3
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pool -o rn -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/bench_prof_pool.log 2>&1 || exit 4
