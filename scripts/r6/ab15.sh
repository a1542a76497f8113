#!/bin/bash
# r6 run 15: unrolled bn_reduce / stem-pool reduction (tests), default bench with the repeated
# labelled image pool (loss must fall), device bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_stem_pool.py tests/test_gpu_shortcut_bn.py tests/test_gpu_kernels.py tests/test_gpu_bnfold.py \
  tests/test_gpu_nnestimator.py -k "pool or shortcut or bn or reduce or nnestimator or stem" -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r6/ab15_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab15_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2 3; do
  $T 300 python -u bench.py > gpurun_out/r6/ab15_fs_$i.log 2>&1 || exit 22
  python3 -c "import json; d=json.loads(open('gpurun_out/r6/ab15_fs_$i.log').read().strip().splitlines()[-1]); print('fs', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
done
$T 300 python -u bench.py --input device > gpurun_out/r6/ab15_dev.log 2>&1 || exit 22
python3 -c "import json; d=json.loads(open('gpurun_out/r6/ab15_dev.log').read().strip().splitlines()[-1]); print('dev', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
