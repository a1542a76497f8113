set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="timeout -s KILL 60 rocprofv3 --kernel-include-regex igemm"
S=analytics-zoo_amd/tools/conv1x1_one.py
for op in fwd dgrad; do
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d gpurun_out/pmc_$op -o a -- python3 $S 56 64 256 $op 5 > gpurun_out/pmc_a_$op.log 2>&1 || exit 1
$P --pmc FETCH_SIZE -d gpurun_out/pmc_$op -o b -- python3 $S 56 64 256 $op 5 > gpurun_out/pmc_b_$op.log 2>&1 || exit 2
$P --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_$op -o c -- python3 $S 56 64 256 $op 5 > gpurun_out/pmc_c_$op.log 2>&1 || exit 3
$P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_CYCLES -d gpurun_out/pmc_$op -o d -- python3 $S 56 64 256 $op 5 > gpurun_out/pmc_d_$op.log 2>&1 || exit 4
done
