#!/bin/bash
# r5 batch 34: new wgrad default (512 workgroups): conv tests + DMA staging A/B x3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad or conv" \
  tests/test_gpu_wgrad256.py tests/test_gpu_resnet50_parity.py > gpurun_out/r5/b34_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b34_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b34_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_DMA=1 $T 200 python -u bench.py > gpurun_out/r5/b34_dma_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b34_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
