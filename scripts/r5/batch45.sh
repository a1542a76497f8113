#!/bin/bash
# r5 batch 45: compact shortcut gradient on an aux stream (overlaps conv2's backward): tests + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_half_resid.py \
  tests/test_gpu_resnet50_parity.py tests/test_gpu_graph_shapes.py > gpurun_out/r5/b45_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b45_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b45_async_$i.log 2>&1 || exit 10
  ZOO_HALF_ASYNC=0 $T 200 python -u bench.py > gpurun_out/r5/b45_sync_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b45_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
