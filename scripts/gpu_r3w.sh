#!/bin/bash
# round-3 batch W: BERT GELU-backward dgrad tile A/B (256x256 vs 128x128 with slice prefetch)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
ZOO_I2_GELU_TILE=1 $T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gelu or linear" > gpurun_out/t_r3w.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3w.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ZOO_I2_GELU_TILE=$v $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_w_${v}_$i.log 2>&1 || exit 5
    echo "bert gelu_tile=$v run $i: $(grep -v amdgpu.ids gpurun_out/bert_w_${v}_$i.log | tail -1 | cut -c1-160)"
  done
done
echo done
