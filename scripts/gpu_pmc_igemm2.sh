#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on the igemm2 / gemm256 / igemm kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc2
timeout -s KILL 90 rocprofv3 -L > /tmp/pmc_list.txt 2>&1; grep -o "SQ_[A-Z_0-9]*\|TCC_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*\|FETCH_SIZE\|WRITE_SIZE" /tmp/pmc_list.txt | sort -u > gpurun_out/pmc2/list.txt
echo "list rc=$?"
ok() {  # keep only counters the list knows
  python3 - "$@" <<'PY'
import sys,re
txt=open('gpurun_out/pmc2/list.txt').read()
print(' '.join(c for c in sys.argv[1:] if re.search(r'\b'+c+r'\b', txt)))
PY
}
PA=$(ok SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS)
PB=$(ok SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE)
echo "PA=$PA"; echo "PB=$PB"
S=analytics-zoo_amd/tools/igemm2_one.py
run() {  # name, args...
  n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "igemm|gemm256" --pmc $PA -d /tmp/pmc2/$n -o a -- python3 $S "$@" > gpurun_out/pmc2/${n}_a.log 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "igemm|gemm256" --pmc $PB -d /tmp/pmc2/$n -o b -- python3 $S "$@" > gpurun_out/pmc2/${n}_b.log 2>&1 || return 2
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "igemm|gemm256" --pmc FETCH_SIZE -d /tmp/pmc2/$n -o c -- python3 $S "$@" > gpurun_out/pmc2/${n}_c.log 2>&1 || return 3
}
run g8k_t5 --gemm 8192,8192,8192 --tile 5 || exit 11
run g8k_g256 --gemm 8192,8192,8192 --gemm256 || exit 12
run c14_t5 --conv 14,256,256,3,1,1 --tile 5 || exit 13
run c14_old --conv 14,256,256,3,1,1 --old || exit 14
run c56_t4 --conv 56,64,64,3,1,1 --tile 4 || exit 15
run c56_old --conv 56,64,64,3,1,1 --old || exit 16
for f in $(find /tmp/pmc2 -name "*.db" | sort); do python3 analytics-zoo_amd/tools/pmc_summary.py $f; done > gpurun_out/pmc2/summary.txt 2>&1; find /tmp/pmc2 -type f | head -50 > gpurun_out/pmc2/files.txt
for f in gpurun_out/pmc2/*_a.log; do echo "== $f"; tail -3 $f; done; du -sh gpurun_out; echo done
