#!/bin/bash
# r5 batch 11: BN-backward prologue fix (deterministic fallback) + kernel-level profile pro vs no-pro
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfold.py > gpurun_out/r5/b11_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r5/b11_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
ZOO_BN_FOLD=1 bash scripts/r5/prof_crit.sh pro > /dev/null || exit 4
ZOO_BN_FOLD=0 bash scripts/r5/prof_crit.sh nopro > /dev/null || exit 5
grep -E "pw_kernel|bn_bwd_apply|bnpro|bnfold" gpurun_out/r5/prof_rn_pro_summary.md | head -30
echo ----
grep -E "pw_kernel|bn_bwd_apply|bnpro|bnfold" gpurun_out/r5/prof_rn_nopro_summary.md | head -30
