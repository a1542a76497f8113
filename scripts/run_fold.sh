set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_wgrad256.py tests/test_gpu_tf_native.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fold.log 2>&1 || exit 1
$T 200 python analytics-zoo_amd/tools/wgrad_bench.py --resnet > gpurun_out/wb_resnet2.log 2>&1 || exit 2
$T 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_fold.log 2>&1 || exit 3
