#!/bin/bash
# r6 run 11: GELU linears store their pre-activation from the GEMM epilogue (tests, BERT A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_gelu_dgrad.py tests/test_gpu_bert_parity.py tests/test_gpu_ibo.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab11_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab11_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PYTHONPATH=$PWD/analytics-zoo_amd:$PYTHONPATH
for i in 1 2 3; do
  for d in False True; do
    $T 300 python3 -u -c "
import sys, runpy
import zoo.ops.conv as C
C._GELU_DUAL = $d
sys.argv = ['bert_train.py', '--batch', '128', '--iters', '20']
runpy.run_path('analytics-zoo_amd/tools/bert_train.py', run_name='__main__')
" > gpurun_out/r6/ab11_bert_dual${d}_$i.log 2>&1 || exit 31
    echo "dual=$d $(tail -1 gpurun_out/r6/ab11_bert_dual${d}_$i.log | cut -c1-110)"
  done
done
