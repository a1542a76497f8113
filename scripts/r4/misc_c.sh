#!/bin/bash
# wgrad256 split-count A/B: whole-network wgrad ms (ResNet-50 b256) and BERT linear shapes per
# ZOO_WGRAD256_WG (target workgroups; fewer = less partial traffic, more M per workgroup)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/misc
for wg in 256 128 64 192; do
  ZOO_WGRAD256_WG=$wg timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops wgrad > gpurun_out/misc/wg_rn_$wg.log 2>&1 || exit 3
  echo "WG=$wg resnet $(tail -1 gpurun_out/misc/wg_rn_$wg.log)"
  ZOO_WGRAD256_WG=$wg timeout -k 10 200 python -u analytics-zoo_amd/tools/wgrad_bench.py > gpurun_out/misc/wg_bert_$wg.log 2>&1 || exit 4
  python3 -c "
import json,sys
for l in open('gpurun_out/misc/wg_bert_$wg.log'):
    if l.startswith('{'):
        r=json.loads(l); print('  bert', r['M'], r['N'], r['K'], r['zoo_wgrad256']['us'], 'us')
"
done
# BERT-base b128: fused residual LayerNorm on / off (same box)
for f in 1 0 1; do
  ZOO_DROP_LN_FUSE=$f timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > gpurun_out/misc/bert_dln$f.log 2>&1 || exit 5
  echo "DROP_LN_FUSE=$f $(tail -1 gpurun_out/misc/bert_dln$f.log)"
done
# int8 / fp8 inference: throughput + top-1 agreement with bf16
timeout -k 10 400 python -u analytics-zoo_amd/tools/quant_bench.py --batch 256 --iters 20 > gpurun_out/misc/quant.log 2>&1 || exit 6
tail -6 gpurun_out/misc/quant.log
