#!/bin/bash
# c3 numerics, kernel trace of the stage-1 3x3 fwd / dgrad, end-to-end bench A/B (ZOO_C3 0 / 1)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c3
TAG=${1:-a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/c3/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
S=analytics-zoo_amd/tools/igemm2_one.py
kt() {
  n=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/c3p/$n -o k -- python3 $S "$@" > gpurun_out/c3/${n}.log 2>&1 || return 1
  f=$(find /tmp/c3p/$n -name "*.db" | head -1)
  echo "$n $(python3 analytics-zoo_amd/tools/prof_summary.py $f 20 x | grep -m1 'c3_kernel\|igemm')"
}
kt fwd_$TAG --conv 56,64,64,3,1,1 || exit 2
kt dgrad_$TAG --conv 56,64,64,3,1,1 --dgrad || exit 3
for i in 1 2; do
  for b in 0 1; do
    ZOO_C3=$b timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/c3/bench_c3${b}_${i}_$TAG.log 2>&1 || exit 4
    echo "c3=$b run=$i $(grep -o '"value": [0-9.]*' gpurun_out/c3/bench_c3${b}_${i}_$TAG.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/c3/bench_c3${b}_${i}_$TAG.log)"
  done
done
