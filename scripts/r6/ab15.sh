#!/bin/bash
# r6 run 15: shortcut BN sums from the consumer epilogue (y2), unrolled reductions (tests), default
# bench with the repeated labelled pool (loss must fall) as a same-box A/B of bn._SC_SUMS
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_stem_pool.py tests/test_gpu_shortcut_bn.py tests/test_gpu_kernels.py tests/test_gpu_bnfold.py \
  tests/test_gpu_nnestimator.py tests/test_gpu_resnet50_parity.py -k "pool or shortcut or bn or reduce or nnestimator or stem or resnet50" \
  -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab15_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab15_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PYTHONPATH=$PWD/analytics-zoo_amd:$PYTHONPATH
run() {  # tag, on
  $T 300 python -u -c "
import sys, runpy
import zoo.ops.bn as B
B._SC_SUMS = $2
sys.argv = ['bench.py']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r6/ab15_$1.log 2>&1 || exit 21
  python3 -c "import json; d=json.loads(open('gpurun_out/r6/ab15_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
}
for i in 1 2 3; do
  run off$i False
  run on$i True
done
