#!/bin/bash
# in-backward optimizer: numerics + end-to-end A/B (ZOO_OPTIM_IN_BWD 1 / 0)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ibo; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ibo.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for s in 1 0; do
    ZOO_OPTIM_IN_BWD=$s timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/rn_i${s}_$i.log 2>&1 || exit 3
    echo "resnet ibo=$s run=$i $(grep -o '"value": [0-9.]*' $O/rn_i${s}_$i.log) $(grep -o '"final_loss": [0-9.]*' $O/rn_i${s}_$i.log)"
  done
done
for i in 1 2; do
  for s in 1 0; do
    ZOO_OPTIM_IN_BWD=$s timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/bert_i${s}_$i.log 2>&1 || exit 4
    echo "bert ibo=$s run=$i $(tail -1 $O/bert_i${s}_$i.log)"
  done
done
