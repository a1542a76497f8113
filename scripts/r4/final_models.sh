#!/bin/bash
# Final-tree numbers for the secondary models: BERT-base b128 step (two runs) and NCF
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/final; mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/bert_$i.log 2>&1 || exit 5
  tail -1 $O/bert_$i.log
done
timeout -k 10 200 python -u bench.py --model ncf > $O/ncf.log 2>&1 || exit 6
tail -1 $O/ncf.log
