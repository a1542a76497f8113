#!/bin/bash
# r5 round-end serving suite: Cluster Serving suite (ResNet-50 + BERT-base), look-ahead worker, full load sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u analytics-zoo_amd/tools/serving_bench.py suite --duration 6 --images 4096 \
  --fractions 0.25,0.5,0.7,0.85,1.0,1.2,1.4 --out gpurun_out/r5/bfinal_suite.json > gpurun_out/r5/bfinal_suite.log 2>&1 || exit 12
grep -h '"bench"' gpurun_out/r5/bfinal_suite.log | cut -c1-330
