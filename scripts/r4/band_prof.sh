#!/bin/bash
# kernel trace + PMC passes of the band tile vs the old per-tap kernels on the stage-1 / 2 3x3 convs
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bandprof
S=analytics-zoo_amd/tools/igemm2_one.py
O=gpurun_out/bandprof
kt() {  # name, env, args...
  n=$1; e=$2; shift 2
  env $e true
  timeout -k 10 120 env $e rocprofv3 --kernel-trace --stats -d /tmp/bp/$n -o k -- python3 $S "$@" > $O/${n}_kt.log 2>&1 || return 1
  f=$(find /tmp/bp/$n -name "*.db" | head -1)
  python3 analytics-zoo_amd/tools/prof_summary.py $f 20 "$n" > $O/${n}_kt.md 2>&1
  grep -m3 "igemm" $O/${n}_kt.md
}
ZOO_I2_BAND=1 kt c56_band ZOO_I2_BAND=1 --conv 56,64,64,3,1,1 || exit 11
kt c56_old ZOO_I2_BAND=0 --conv 56,64,64,3,1,1 || exit 12
kt c56_band_dg ZOO_I2_BAND=1 --conv 56,64,64,3,1,1 --dgrad || exit 13
kt c28_band ZOO_I2_BAND=1 --conv 28,128,128,3,1,1 || exit 14
kt c28_band_w ZOO_I2_BAND_TILE=10 --conv 28,128,128,3,1,1 || exit 15
kt c28_old ZOO_I2_BAND=0 --conv 28,128,128,3,1,1 || exit 16
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
PB="FETCH_SIZE TCC_HIT_sum"
PC="WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_VALU"
for p in A B C; do
  eval cs=\$P$p
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "igemm" --pmc $cs -d /tmp/bpp/$p -o p -- python3 $S --conv 56,64,64,3,1,1 --iters 5 > $O/pmc_$p.log 2>&1 || { echo "pmc $p failed"; tail -3 $O/pmc_$p.log; break; }
done
for f in $(find /tmp/bpp -name "*.db" | sort); do python3 analytics-zoo_amd/tools/pmc_summary.py $f; done > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt | head -60
