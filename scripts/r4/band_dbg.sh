#!/bin/bash
# band kernel bottleneck hunt: kernel time with parts switched off (ZOO_I2_DBG bits)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/banddbg
S=analytics-zoo_amd/tools/igemm2_one.py
O=gpurun_out/banddbg
for d in 0 1 2 3 4 6 8 10 12 14; do
  timeout -k 10 120 env ZOO_I2_DBG=$d rocprofv3 --kernel-trace --stats -d /tmp/bd/$d -o k -- python3 $S --conv 56,64,64,3,1,1 > $O/d${d}.log 2>&1 || exit 1
  f=$(find /tmp/bd/$d -name "*.db" | head -1)
  echo "dbg=$d $(python3 analytics-zoo_amd/tools/prof_summary.py $f 20 x | grep -m1 igemm2)"
done
