#!/bin/bash
# r5 batch 35: wgrad DMA staging on by default (tests) + wgrad256 conv split target sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad or conv" \
  tests/test_gpu_wgrad256.py tests/test_gpu_resnet50_parity.py tests/test_gpu_zoo_kernels.py > gpurun_out/r5/b35_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b35_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b35_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD256_CONV_WG=64 $T 200 python -u bench.py > gpurun_out/r5/b35_cw64_$i.log 2>&1 || exit 11
  ZOO_WGRAD256_CONV_WG=96 $T 200 python -u bench.py > gpurun_out/r5/b35_cw96_$i.log 2>&1 || exit 12
  ZOO_WGRAD256_CONV_WG=192 $T 200 python -u bench.py > gpurun_out/r5/b35_cw192_$i.log 2>&1 || exit 13
done
for f in gpurun_out/r5/b35_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
