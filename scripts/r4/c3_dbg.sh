#!/bin/bash
# c3 bottleneck hunt: kernel time with parts switched off (ZOO_C3_DBG bits), plus PMC
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c3dbg
S=analytics-zoo_amd/tools/igemm2_one.py
O=gpurun_out/c3dbg
for d in 0 1 2 4 8 3 6 9 14 15; do
  timeout -k 10 120 env ZOO_C3_DBG=$d rocprofv3 --kernel-trace --stats -d /tmp/cd/$d -o k -- python3 $S --conv 56,64,64,3,1,1 > $O/d${d}.log 2>&1 || exit 1
  f=$(find /tmp/cd/$d -name "*.db" | head -1)
  echo "dbg=$d $(python3 analytics-zoo_amd/tools/prof_summary.py $f 20 x | grep -m1 c3_kernel)"
done
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS"
PB="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
PC="FETCH_SIZE TCC_HIT_sum"
PD="WRITE_SIZE TCC_EA0_WRREQ_sum"
for p in A B C D; do
  eval cs=\$P$p
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "c3_kernel" --pmc $cs -d /tmp/cdp/$p -o p -- python3 $S --conv 56,64,64,3,1,1 --iters 5 > $O/pmc_$p.log 2>&1 || { echo "pmc $p failed"; tail -3 $O/pmc_$p.log; }
done
for f in $(find /tmp/cdp -name "*.db" | sort); do python3 analytics-zoo_amd/tools/pmc_summary.py $f; done > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt
