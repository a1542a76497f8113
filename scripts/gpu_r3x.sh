#!/bin/bash
# round-3 batch X: full GPU suite + smoke + bench A/B (EPI 2 batching with the gated prologue prefetch, igemm BN 128)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r3x_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3x_full.log; [ $rc = 0 ] || exit 1
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_x.log 2>&1 || exit 2
tail -1 gpurun_out/smoke_x.log
for i in 1 2; do
  for v in "0 0" "1 0" "1 128"; do
    set -- $v
    ZOO_EPI2_BATCH=$1 ZOO_IGEMM_BN=$2 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_x_$1_$2_$i.log 2>&1 || exit 3
    echo "epi2_batch=$1 igemm_bn=$2 run $i: $(tail -1 gpurun_out/bench_x_$1_$2_$i.log | cut -c1-150)"
  done
done
echo done
