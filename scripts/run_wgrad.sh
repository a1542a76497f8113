set -o pipefail
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet50_parity.py -x -q --timeout 200 --timeout-method thread -k "conv or resnet or parity or linear or deterministic or partial" > gpurun_out/pytest_wgrad.log 2>&1 || exit 1
$T 200 python analytics-zoo_amd/tools/conv_sweep.py --ops wgrad --detail > gpurun_out/sweep_wgrad_new.log 2>&1 || exit 2
ZOO_WGRAD_BM64=0 $T 200 python analytics-zoo_amd/tools/conv_sweep.py --ops wgrad --detail > gpurun_out/sweep_wgrad_bm128.log 2>&1 || exit 3
$T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_wgrad.log 2>&1 || exit 4
