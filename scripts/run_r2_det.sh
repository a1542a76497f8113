set -o pipefail
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_resnet50_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || exit 1
for m in "0 0" "1 0" "0 1" "1 1"; do set -- $m
  ZOO_STATS_PARTIAL=$1 ZOO_WGRAD_PARTIAL=$2 $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_sp$1_wp$2.log 2>&1 || exit 2
done
ZOO_DETERMINISTIC=1 $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_det1.log 2>&1 || exit 3
ZOO_DETERMINISTIC=1 $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_det2.log 2>&1 || exit 4
