#!/bin/bash
# band-tile numerics, per-shape conv sweep and end-to-end bench A/B (ZOO_I2_BAND 0 / 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-band}
timeout -k 10 300 python -u -m pytest tests/test_gpu_igemm2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_igemm2_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_igemm2_$TAG.log
[ $rc -eq 0 ] || exit $rc
for b in 0 1; do
  ZOO_I2_BAND=$b timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops fwd,dgrad --detail > gpurun_out/sweep_band${b}_$TAG.log 2>&1 || exit 3
  tail -1 gpurun_out/sweep_band${b}_$TAG.log
done
for i in 1 2; do
  for b in 0 1; do
    ZOO_I2_BAND=$b timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_band${b}_${i}_$TAG.log 2>&1 || exit 4
    echo "band=$b run=$i $(grep -o '"value": [0-9.]*' gpurun_out/bench_band${b}_${i}_$TAG.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/bench_band${b}_${i}_$TAG.log)"
  done
done
