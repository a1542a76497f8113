#!/bin/bash
# r5 batch 15: BERT-base training under hipGraph with the runtime's graph-queue switches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 > gpurun_out/r5/b15_bert_eager.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b15_bert_eager.log
$T 200 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --graph > gpurun_out/r5/b15_bert_graph.log 2>&1 || exit 4
tail -1 gpurun_out/r5/b15_bert_graph.log
for q in 2 4 8; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q $T 200 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --graph > gpurun_out/r5/b15_bert_graph_q$q.log 2>&1 || exit 5
  echo "queues $q: $(tail -1 gpurun_out/r5/b15_bert_graph_q$q.log)"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $T 200 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --graph > gpurun_out/r5/b15_bert_graph_nopkt.log 2>&1 || exit 6
echo "no packet capture: $(tail -1 gpurun_out/r5/b15_bert_graph_nopkt.log)"
