#!/bin/bash
# r5 batch 29: unsigned (offset-coded) int8 activations: kernel tests + quant bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_qconv.py tests/test_quant.py \
  > gpurun_out/r5/b29_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b29_tests.log
[ $rc -eq 0 ] || exit $rc
$T 800 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/b29_quant.log 2>&1 || exit 7
tail -1 gpurun_out/r5/b29_quant.log | python3 -c '
import sys, json
r = json.loads(sys.stdin.read())
for k, v in r.items():
    if ("top1_agree" in k and "margin" not in k) or "rowcos" in k or "task_acc" in k or "img_s" in k:
        print(k, v)'
