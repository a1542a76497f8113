#!/bin/bash
# weight-gradient side stream: numerics (ResNet / BERT parity, engine tests) + end-to-end A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ws; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet50_parity.py tests/test_gpu_bert_parity.py tests/test_gpu_ddp.py tests/test_gpu_round3.py \
  -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for s in 1 0; do
    ZOO_WGRAD_STREAM=$s timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/rn_s${s}_$i.log 2>&1 || exit 3
    echo "resnet stream=$s run=$i $(grep -o '"value": [0-9.]*' $O/rn_s${s}_$i.log) $(grep -o '"final_loss": [0-9.]*' $O/rn_s${s}_$i.log)"
  done
done
for s in 1 0; do
  ZOO_WGRAD_STREAM=$s timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/bert_s$s.log 2>&1 || exit 4
  echo "bert stream=$s $(tail -1 $O/bert_s$s.log)"
done
