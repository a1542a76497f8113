#!/bin/bash
# c3 quick loop: numerics, kernel trace of fwd / dgrad, stamp shares
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c3
TAG=${1:-q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/c3/pytest_$TAG.log
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
ZOO_C3_STAMPS=1 timeout -k 10 120 python3 analytics-zoo_amd/tools/c3_stamps.py || exit 4
