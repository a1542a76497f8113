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
