#!/bin/bash
# r6 run 35: forward row groups at >= 64k pixels (backward K-split) -- tests, 32^3 A/B vs forward K-split
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_convlstm_seq.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab35_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6/ab35_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  $T 300 python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes loop,fused --iters 5 >> gpurun_out/r6/ab35_cl3d.log 2>&1 || exit 42
done
grep bench gpurun_out/r6/ab35_cl3d.log | cut -c1-260
$T 300 python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --hw 16 --modes loop,fused --iters 10 >> gpurun_out/r6/ab35_cl3d.log 2>&1 || exit 43
grep bench gpurun_out/r6/ab35_cl3d.log | cut -c1-200
