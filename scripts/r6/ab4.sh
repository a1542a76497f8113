#!/bin/bash
# r6 run 4: captured-step tests (batched filter flip under capture), ResNet-50 step trace with every
# round-6 fusion on, BERT graph/eager timing + graph trace, ConvLSTM 2-D/3-D bench, serving suite x3
# with the sharded store + GC freeze
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ibo.py tests/test_gpu_graph_shapes.py tests/test_gpu_kernels.py -k "ibo or graph or capture or serving or predict or jpeg" -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab4_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 4 ] || [ $rc -eq 5 ] || exit $rc
rm -rf /tmp/prof_rn
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 bench.py --input device --steps 8 --warmup 3 > gpurun_out/r6/ab4_prof_rn.log 2>&1 || exit 8
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r6/ab4_prof_rn_step.md 2>&1
tail -34 gpurun_out/r6/ab4_prof_rn_step.md
for i in 1 2; do
  $T 300 python3 -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --graph > gpurun_out/r6/ab4_bert_graph$i.log 2>&1 || exit 31
  tail -1 gpurun_out/r6/ab4_bert_graph$i.log | cut -c1-300
done
rm -rf /tmp/prof_bert_graph
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert_graph -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 --graph > gpurun_out/r6/ab4_prof_bert_graph.log 2>&1 || exit 32
DB=$(find /tmp/prof_bert_graph -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB softmax_xent 13 --critical > gpurun_out/r6/ab4_prof_bert_graph_step.md 2>&1
tail -12 gpurun_out/r6/ab4_prof_bert_graph_step.md
for d in 2 3; do
  $T 300 python3 -u analytics-zoo_amd/tools/convlstm_bench.py --dims $d --T 16 > gpurun_out/r6/ab4_convlstm_${d}d.log 2>&1 || exit 41
  tail -2 gpurun_out/r6/ab4_convlstm_${d}d.log | cut -c1-400
done
bash scripts/r6/serving.sh
