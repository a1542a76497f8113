#!/bin/bash
# r6 run 18: block-output prologue at the stage-1 -> stage-2 transition (tests + same-box A/B), and
# a re-A/B of the inner-unit forward prologue (FWD_PRO) on the round-6 kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_fwd_pro.py tests/test_gpu_resnet50_parity.py tests/test_gpu_shortcut_bn.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab18_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab18_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PYTHONPATH=$PWD/analytics-zoo_amd:$PYTHONPATH
run() {  # tag, down, fwdpro
  $T 300 python -u -c "
import sys, runpy
import zoo.models.image.resnet as R
R.FWD_PRO_RES_DOWN = $2
R.FWD_PRO = $3
sys.argv = ['bench.py']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r6/ab18_$1.log 2>&1 || exit 21
  python3 -c "import json; d=json.loads(open('gpurun_out/r6/ab18_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
}
for i in 1 2 3; do
  run off$i False False
  run down$i True False
  run downfp$i True True
done
