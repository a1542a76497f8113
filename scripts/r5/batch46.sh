#!/bin/bash
# r5 batch 46: BERT-base b128 s128 training -- wgrad256 split target sweep on the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > gpurun_out/r5/b46_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD256_WG=128 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > gpurun_out/r5/b46_wg128_$i.log 2>&1 || exit 11
  ZOO_WGRAD256_WG=512 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > gpurun_out/r5/b46_wg512_$i.log 2>&1 || exit 12
done
for f in gpurun_out/r5/b46_*_?.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"host_ms_per_step": [0-9.]*' $f)"; done
