#!/bin/bash
# BERT: attention backward (persistent dK/dV + 4-wave dQ), bias sums and LayerNorm folds on the side stream
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/bert2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert_parity.py tests/test_gpu_drop_ln.py tests/test_gpu_residual_grad.py \
  tests/test_gpu_ibo.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 2
for i in 1 2; do
  timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/new_$i.log 2>&1 || exit 3
  echo "new run=$i $(tail -1 $O/new_$i.log)"
  ZOO_ATTN_PERSIST=0 ZOO_ATTN_DQ4=0 timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/oldattn_$i.log 2>&1 || exit 4
  echo "old-attn run=$i $(tail -1 $O/oldattn_$i.log)"
done
