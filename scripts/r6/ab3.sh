#!/bin/bash
# r6 A/B 3: block-output prologue (FWD_PRO_RES) numerics + same-box A/B; isolated BERT GEMMs;
# Cluster Serving suite x3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_fwd_pro.py tests/test_gpu_resnet50_parity.py tests/test_gpu_native_nets.py \
  tests/test_gpu_bnfold.py tests/test_gpu_half_resid.py -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/ab3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab3_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, on
  $T 300 python -u -c "
import sys, runpy
import zoo.models.image.resnet as R
R.FWD_PRO_RES = $2
sys.argv = ['bench.py', '--input', 'device']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r6/ab3_$1.log 2>&1 || exit 21
  python3 -c "import json; d=json.loads(open('gpurun_out/r6/ab3_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
}
export PYTHONPATH=$PWD/analytics-zoo_amd:$PYTHONPATH
for i in 1 2; do
  run off$i False
  run on$i True
done
$T 300 python -u bench.py > gpurun_out/r6/ab3_default_fs.log 2>&1 || exit 22
tail -1 gpurun_out/r6/ab3_default_fs.log | cut -c1-160
$T 300 python3 -u analytics-zoo_amd/tools/gemm_bench.py --bert > gpurun_out/r6/ab3_gemm_bert.log 2>&1 || exit 23
tail -12 gpurun_out/r6/ab3_gemm_bert.log
bash scripts/r6/serving.sh
