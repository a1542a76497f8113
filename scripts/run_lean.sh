set -o pipefail
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "conv or resnet or parity or linear" > gpurun_out/pytest_lean.log 2>&1 || exit 1
$T 120 python analytics-zoo_amd/tools/conv1x1_probe.py > gpurun_out/probe_lean.log 2>&1 || exit 2
$T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_lean.log 2>&1 || exit 3
ZOO_IGEMM_LEAN=0 $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nolean.log 2>&1 || exit 4
