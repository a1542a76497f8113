set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_nets.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rn.log 2>&1 || exit 1
$T 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_rn.log 2>&1 || exit 2
ZOO_WGRAD256=0 $T 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_rn_off.log 2>&1 || exit 3
