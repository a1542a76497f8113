set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_qconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_q8.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/quant_bench.py --batch 256 --iters 20 > gpurun_out/quant_bench.log 2>&1 || exit 2
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8 -o q8 -- python3 analytics-zoo_amd/tools/quant_bench.py --batch 256 --iters 10 --no-dynamic > gpurun_out/prof_q8.log 2>&1 || exit 3
