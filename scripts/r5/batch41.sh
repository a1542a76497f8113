#!/bin/bash
# r5 batch 41: stem weight gradient pipelined into the pool backward (StemWgrad): tests + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stem_pool.py \
  tests/test_gpu_pw_stem.py tests/test_gpu_resnet50_parity.py > gpurun_out/r5/b41_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b41_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b41_pipe_$i.log 2>&1 || exit 10
  ZOO_STEM_PIPE=0 $T 200 python -u bench.py > gpurun_out/r5/b41_serial_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b41_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
