#!/bin/bash
# r5 batch 10: BN-backward prologue in the 1x1 dgrad (tests, parity, same-box A/B), dropout under
# graph, quant bench with the partly-trained / diverged models
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfold.py \
  "tests/test_gpu_ibo.py::test_graph_replay_draws_fresh_dropout_masks" tests/test_gpu_resnet50_parity.py \
  tests/test_gpu_pw.py tests/test_gpu_kernels.py -k "bnfold or prologue or dropout or resnet or pw" > gpurun_out/r5/b10_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5/b10_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b10_pro_$i.log 2>&1 || exit 10
  ZOO_BN_FOLD=0 $T 200 python -u bench.py > gpurun_out/r5/b10_nopro_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b10_{pro,nopro}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
$T 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_native_nets.py -k "layer_parity" -s \
  > gpurun_out/r5/b10_parity.log 2>&1
rc=$?
grep -E "layers|passed|failed" gpurun_out/r5/b10_parity.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 600 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/b10_quant.log 2>&1 || exit 7
tail -1 gpurun_out/r5/b10_quant.log
