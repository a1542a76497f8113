#!/bin/bash
# r6 run 31: two-launch mean softmax-xent + one-pass backward -- tests, then bench A/B (3 pairs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nnestimator.py tests/test_gpu_resnet50_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab31_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab31_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in False True; do
    $T 400 python -u scripts/r6/bench_ab.py zoo.ops.loss _XENT_MEAN $v > gpurun_out/r6/ab31_${v}_$i.log 2>&1 || exit 46
    echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/r6/ab31_${v}_$i.log)"
  done
done
