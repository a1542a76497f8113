#!/bin/bash
# quick band A/B: kernel trace of the two band shapes (fwd / dgrad) and the conv sweep
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bandq
S=analytics-zoo_amd/tools/igemm2_one.py
O=gpurun_out/bandq
TAG=${1:-q}
kt() {
  n=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/bq/$n -o k -- python3 $S "$@" > $O/${n}.log 2>&1 || return 1
  f=$(find /tmp/bq/$n -name "*.db" | head -1)
  echo "$n $(python3 analytics-zoo_amd/tools/prof_summary.py $f 20 x | grep -m1 'igemm')"
}
kt c56f_$TAG --conv 56,64,64,3,1,1 || exit 1
kt c56d_$TAG --conv 56,64,64,3,1,1 --dgrad || exit 2
kt c28f_$TAG --conv 28,128,128,3,1,1 || exit 3
kt c28d_$TAG --conv 28,128,128,3,1,1 --dgrad || exit 4
ZOO_I2_BAND_TILE=10 kt c28fw_$TAG --conv 28,128,128,3,1,1 || exit 5
kt c14f_$TAG --conv 14,256,256,3,1,1 || exit 6
