#!/bin/bash
# r5 batch 53: serving latency tail with the async rings warmed (ResNet-50, 0.7 / 0.85 load)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for sw in 0; do
  ZOO_SERVING_SWITCH_MS=$sw $T 400 python -u analytics-zoo_amd/tools/serving_bench.py suite --models resnet50 --duration 6 \
    --images 4096 --fractions 0.7,0.85,0.7,0.85,1.0 > gpurun_out/r5/b53_sw$sw.log 2>&1 || exit 12
  echo "switch $sw ms"; grep -h '"bench"' gpurun_out/r5/b53_sw$sw.log | python3 -c '
import sys, json
for l in sys.stdin:
    r = json.loads(l)
    print(r.get("load_fraction_of_capacity", "cap"), r.get("achieved_throughput", r.get("drain_throughput")), r.get("p50_ms"), r.get("p90_ms"), r.get("p99_ms"))'
done
