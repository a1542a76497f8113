#!/bin/bash
# round-3 batch Y: LayerNorm residual-gradient add (tests + BERT A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_residual_grad.py tests/test_gpu_gelu_dgrad.py tests/test_gpu_kernels.py -k "residual or gelu or layernorm or layer_norm" > gpurun_out/t_r3y.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3y.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ZOO_LN_GRAD_ADD=$v $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_y_${v}_$i.log 2>&1 || exit 5
    echo "bert ln_grad_add=$v run $i: $(grep -v amdgpu.ids gpurun_out/bert_y_${v}_$i.log | tail -1 | cut -c1-160)"
  done
done
echo done
