#!/bin/bash
# r5 batch 28: SmoothQuant-style activation scale split for the int8 / fp8 ResNet twins
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_qconv.py -k "int8_resnet_tracks or mse" \
  > gpurun_out/r5/b28_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b28_tests.log
[ $rc -eq 0 ] || exit $rc
$T 700 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/b28_quant.log 2>&1 || exit 7
tail -1 gpurun_out/r5/b28_quant.log | python3 -c '
import sys, json
r = json.loads(sys.stdin.read())
for k, v in r.items():
    if "top1_agree" in k and "margin" not in k or "rowcos" in k or "task_acc" in k:
        print(k, v)'
