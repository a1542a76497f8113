#!/bin/bash
# r5 batch 57: serving GPU tests after the last serving changes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py -k "serving or inference or jpeg" \
  > gpurun_out/r5/b57_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b57_tests.log
exit $rc
