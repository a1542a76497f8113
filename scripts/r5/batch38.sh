#!/bin/bash
# r5 batch 38: the compact shortcut data gradient on pw.hip (512-deep reduction) A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
ZOO_COMPACT_DGRAD_KMAX=512 $T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_half_resid.py \
  > gpurun_out/r5/b38_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b38_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b38_def_$i.log 2>&1 || exit 10
  ZOO_COMPACT_DGRAD_KMAX=512 $T 200 python -u bench.py > gpurun_out/r5/b38_k512_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b38_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
