#!/bin/bash
# r5 batch 9: ConvLSTM sequences issued from C++ (tests + bench); kernel-level profile of the
# BN-backward fold vs the materialised BN backward
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_convlstm_seq.py \
  tests/test_gpu_keras_native.py -k "ConvLSTM or convlstm" > gpurun_out/r5/b9_convlstm.log 2>&1
rc=$?
tail -4 gpurun_out/r5/b9_convlstm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b9_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b9_convlstm_bench.log
ZOO_BN_FOLD=1 bash scripts/r5/prof_crit.sh fold > /dev/null || exit 4
ZOO_BN_FOLD=0 bash scripts/r5/prof_crit.sh nofold > /dev/null || exit 5
grep -E "bnfold|bn_bwd_apply|igemm|pw_kernel|wgrad|bn_reduce" gpurun_out/r5/prof_rn_fold_summary.md | head -30
echo ----
grep -E "bnfold|bn_bwd_apply|igemm|pw_kernel|wgrad|bn_reduce" gpurun_out/r5/prof_rn_nofold_summary.md | head -30
