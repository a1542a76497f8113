#!/bin/bash
# r6 run 12: NCF records/s (bench default: native comm + captured step), BERT eager / graph with the
# GELU dual store, Cluster Serving suite (GC collect-once variant), smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 300 python -u bench.py --model ncf > gpurun_out/r6/ab12_ncf_$i.log 2>&1 || exit 21
  tail -1 gpurun_out/r6/ab12_ncf_$i.log | cut -c1-400
done
$T 300 python -u bench.py --model ncf --force-comm > gpurun_out/r6/ab12_ncf_forcecomm.log 2>&1 || exit 22
tail -1 gpurun_out/r6/ab12_ncf_forcecomm.log | cut -c1-400
for m in "" "--graph"; do
  $T 300 python3 -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 $m > gpurun_out/r6/ab12_bert$m.log 2>&1 || exit 31
  tail -1 gpurun_out/r6/ab12_bert$m.log | cut -c1-300
done
$T 600 python -u analytics-zoo_amd/tools/serving_bench.py suite --duration 6 --images 16384 \
  --fractions 0.5,0.7,0.85,1.0,1.2 --out gpurun_out/r6/ab12_serving.json > gpurun_out/r6/ab12_serving.log 2>&1 || exit 12
grep -h '"bench"' gpurun_out/r6/ab12_serving.log | cut -c1-200
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/ab12_smoke.log 2>&1 || exit 13
tail -1 gpurun_out/r6/ab12_smoke.log
