set -o pipefail
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet50_parity.py -x -q --timeout 200 --timeout-method thread -k "conv or resnet or parity or deterministic or partial" > gpurun_out/pytest_wgrad.log 2>&1 || exit 1
for mb in 0 4 16 64; do
ZOO_WGRAD_PARTIAL_MB=$mb $T 200 python analytics-zoo_amd/tools/conv_sweep.py --ops wgrad --detail > gpurun_out/sweep_wgrad_mb$mb.log 2>&1 || exit 2
done
$T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_wgrad.log 2>&1 || exit 4
ZOO_WGRAD_PARTIAL_MB=0 $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_wgrad_mb0.log 2>&1 || exit 5
