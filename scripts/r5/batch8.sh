#!/bin/bash
# r5 batch 8: one-launch-per-step ConvLSTM2D/3D; BN-backward fold (kernels + model parity) and its A/B; dropout-under-graph and the
# tie-masked per-layer parity re-checked
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_convlstm_seq.py \
  tests/test_gpu_keras_native.py -k "ConvLSTM or convlstm" > gpurun_out/r5/b8_convlstm.log 2>&1
rc=$?
tail -4 gpurun_out/r5/b8_convlstm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b8_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b8_convlstm_bench.log
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfold.py \
  "tests/test_gpu_ibo.py::test_graph_replay_draws_fresh_dropout_masks" tests/test_gpu_resnet50_parity.py \
  tests/test_gpu_kernels.py -k "bnfold or dropout or resnet" > gpurun_out/r5/b8_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5/b8_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_native_nets.py -k "layer_parity" -s \
  > gpurun_out/r5/b8_parity.log 2>&1
rc=$?
grep -E "layers|passed|failed" gpurun_out/r5/b8_parity.log | tail -14
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b8_fold_$i.log 2>&1 || exit 10
  ZOO_BN_FOLD=0 $T 200 python -u bench.py > gpurun_out/r5/b8_nofold_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b8_{fold,nofold}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
