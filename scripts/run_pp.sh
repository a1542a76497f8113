set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_wgrad256.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pp.log 2>&1 || exit 1
ZOO_W256_PINGPONG=0 $T 200 python analytics-zoo_amd/tools/wgrad_bench.py --more > gpurun_out/wb_pp0.log 2>&1 || exit 2
ZOO_W256_PINGPONG=1 $T 200 python analytics-zoo_amd/tools/wgrad_bench.py --more > gpurun_out/wb_pp1.log 2>&1 || exit 3
