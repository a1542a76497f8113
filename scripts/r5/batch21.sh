#!/bin/bash
# r5 batch 21: serving look-ahead (predict_async) + persistent JPEG decode pool: tests + suite A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "inference or serving or jpeg" > gpurun_out/r5/b21_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b21_tests.log
[ $rc -eq 0 ] || exit $rc
for mode in 1 0; do
  ZOO_SERVING_ASYNC=$mode $T 400 python -u analytics-zoo_amd/tools/serving_bench.py suite --models resnet50 \
    --duration 5 --fractions 0.5,0.7,0.85,1.0,1.2 > gpurun_out/r5/b21_suite_async$mode.log 2>&1 || exit 12
  grep -h '"bench"' gpurun_out/r5/b21_suite_async$mode.log | cut -c1-400
done
