set -o pipefail
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_resnet50_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ddp.log 2>&1 || exit 1
$T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit 2
$T 120 python bench.py --steps 20 --warmup 5 --force-comm > gpurun_out/bench_forcecomm.log 2>&1 || exit 3
$T 120 python bench.py --steps 20 --warmup 5 --sharded > gpurun_out/bench_sharded.log 2>&1 || exit 4
$T 120 python bench.py --steps 20 --warmup 5 --sharded --grad-compression bf16 > gpurun_out/bench_sharded_bf16.log 2>&1 || exit 5
$T 120 python bench.py --model ncf --steps 50 --warmup 10 > gpurun_out/bench_ncf.log 2>&1 || exit 6
