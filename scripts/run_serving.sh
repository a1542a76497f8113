set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_serving.py tests/test_gpu_kernels.py -k "serving" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_serving.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/serving_bench.py e2e --images 4096 --batch 64 --drain > gpurun_out/serving_e2e_r2d.log 2>&1 || exit 2
$T 300 python analytics-zoo_amd/tools/serving_bench.py e2e --images 8192 --batch 64 >> gpurun_out/serving_e2e_r2d.log 2>&1 || exit 3
ZOO_SERVING_DECODE_PROCS=14 $T 300 python analytics-zoo_amd/tools/serving_bench.py e2e --images 8192 --batch 128 --drain >> gpurun_out/serving_e2e_r2d.log 2>&1 || exit 4
ZOO_SERVING_DECODE_PROCS=14 $T 300 python analytics-zoo_amd/tools/serving_bench.py e2e --images 8192 --batch 128 --producers 6 >> gpurun_out/serving_e2e_r2d.log 2>&1 || exit 5
