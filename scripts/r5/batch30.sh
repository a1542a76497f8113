#!/bin/bash
# r5 batch 30: unsigned int8 activations (tests + quant bench) and the half-resolution shortcut
# gradient (tests + bench A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_half_resid.py \
  tests/test_gpu_resnet50_parity.py tests/test_gpu_qconv.py tests/test_quant.py > gpurun_out/r5/b30_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b30_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b30_half_$i.log 2>&1 || exit 10
  ZOO_HALF_RESID=0 $T 200 python -u bench.py > gpurun_out/r5/b30_full_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b30_{half,full}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
$T 800 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/b30_quant.log 2>&1 || exit 7
tail -1 gpurun_out/r5/b30_quant.log | python3 -c '
import sys, json
r = json.loads(sys.stdin.read())
for k, v in r.items():
    if (("top1_agree" in k and "margin" not in k) or "rowcos" in k or "task_acc" in k or "img_s" in k) and "clip" not in k and "mse" not in k:
        print(k, v)'
