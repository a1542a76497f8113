#!/bin/bash
# r6 Cluster Serving suite x3 (ResNet-50 + BERT-base): honest ceiling (back-to-back predict_async),
# slowest-1 % batch stage breakdown at every load
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 600 python -u analytics-zoo_amd/tools/serving_bench.py suite --duration 6 --images 16384 \
    --fractions 0.5,0.7,0.85,1.0,1.2 --out gpurun_out/r6/serving_suite_$i.json > gpurun_out/r6/serving_suite_$i.log 2>&1 || exit 12
  grep -h '"bench"' gpurun_out/r6/serving_suite_$i.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if d['bench']=='cluster-serving-capacity': print('cap', d['model'], d['drain_throughput'], d['model_only_throughput'], d['model_only_sync_throughput'], d['drain_over_model'])
    else: print(d['model'][:9], d['load_fraction_of_capacity'], d['achieved_throughput'], d['p50_ms'], d['p90_ms'], d['p99_ms'], d['achieved_over_model'], json.dumps((d.get('rank0_slowest_batches') or {}).get('slowest_mean_ms')))
"
done
