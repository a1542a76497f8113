#!/bin/bash
# PMC passes (kernel-trace only, one counter group per run) on the 3x3 conv kernels of ResNet stage 1/2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc4
timeout -s KILL 90 rocprofv3 -L > /tmp/pmc_list.txt 2>&1; grep -o "SQ_[A-Z_0-9]*\|TCC_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|TA_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*\|FETCH_SIZE\|WRITE_SIZE" /tmp/pmc_list.txt | sort -u > gpurun_out/pmc4/list.txt
ok() {
  python3 - "$@" <<'PY'
import sys,re
txt=open('gpurun_out/pmc4/list.txt').read()
print(' '.join(c for c in sys.argv[1:] if re.search(r'\b'+c+r'\b', txt)))
PY
}
PA=$(ok SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA)
PB=$(ok SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE)
PC=$(ok TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TA_FLAT_READ_WAVEFRONTS_sum)
echo "PA=$PA"; echo "PB=$PB"; echo "PC=$PC"
S=analytics-zoo_amd/tools/igemm2_one.py
run() {
  n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "igemm" --pmc $PA -d /tmp/pmc4/$n -o a -- python3 $S "$@" > gpurun_out/pmc4/${n}_a.log 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "igemm" --pmc $PB -d /tmp/pmc4/$n -o b -- python3 $S "$@" > gpurun_out/pmc4/${n}_b.log 2>&1 || return 2
  if [ -n "$PC" ]; then timeout -s KILL 120 rocprofv3 --kernel-include-regex "igemm" --pmc $PC -d /tmp/pmc4/$n -o c -- python3 $S "$@" > gpurun_out/pmc4/${n}_c.log 2>&1 || return 3; fi
}
run c56_old --conv 56,64,64,3,1,1 --old || exit 15
run c56_t4 --conv 56,64,64,3,1,1 --tile 4 || exit 16
run c28_old --conv 28,128,128,3,1,1 --old || exit 17
run c28_t1 --conv 28,128,128,3,1,1 --tile 1 || exit 18
for f in $(find /tmp/pmc4 -name "*.db" | sort); do echo "## $f"; python3 analytics-zoo_amd/tools/pmc_summary.py $f; done > gpurun_out/pmc4/summary.txt 2>&1
tail -60 gpurun_out/pmc4/summary.txt
