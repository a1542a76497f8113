#!/bin/bash
# round-3 batch M: implicit-GEMM conv weight gradient on wgrad256 (tests, per-shape A/B, bench A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > gpurun_out/t_r3m.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 gpurun_out/t_r3m.log; [ $rc = 0 ] || exit 1
for c in 0 256 128 64; do
  ZOO_WGRAD256_CONV_COUT=$c $T 200 python -u analytics-zoo_amd/tools/wgrad_bench.py --conv > gpurun_out/wconv_$c.log 2>&1 || exit 2
  echo "== cout>=$c"; grep -v amdgpu.ids gpurun_out/wconv_$c.log | cut -c1-200
done
for i in 1 2; do
  for c in 0 256; do
    ZOO_WGRAD256_CONV_COUT=$c $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_m_${c}_$i.log 2>&1 || exit 3
    echo "bench cout>=$c run $i: $(grep '"metric"' gpurun_out/bench_m_${c}_$i.log | cut -c1-120)"
  done
done
echo done
