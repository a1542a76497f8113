#!/bin/bash
# round-3 batch AA: GELU-dgrad bias sums from the per-step arena (tests + BERT timing)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gelu_dgrad.py tests/test_gpu_residual_grad.py > gpurun_out/t_r3aa.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t_r3aa.log; [ $rc = 0 ] || exit 1
for i in 1 2 3; do
  $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_aa_$i.log 2>&1 || exit 5
  echo "bert run $i: $(grep -v amdgpu.ids gpurun_out/bert_aa_$i.log | tail -1 | cut -c1-160)"
done
echo done
