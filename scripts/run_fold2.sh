set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_nets.py tests/test_gpu_wgrad256.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fold2.log 2>&1 || exit 1
$T 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_fold2.log 2>&1 || exit 3
