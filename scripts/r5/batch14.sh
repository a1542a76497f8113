#!/bin/bash
# r5 batch 14: native comm layer tests (world 1); critical-path profile with the prologue on;
# ConvLSTM kernel profile with LDS weights
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm_native.py tests/test_gpu_ddp.py > gpurun_out/r5/b14_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r5/b14_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r5/prof_crit.sh pro2 > /dev/null || exit 4
tail -32 gpurun_out/r5/prof_rn_pro2_step.md
$T 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cl -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --iters 3 > gpurun_out/r5/b14_prof_cl.log 2>&1 || exit 12
DB=$(find /tmp/prof_cl -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM2D T=32 bench (3 modes, 5 iters each)" > gpurun_out/r5/b14_prof_cl_summary.md 2>&1
grep -E "convlstm|lstm_step|igemm|wgrad" gpurun_out/r5/b14_prof_cl_summary.md | head -12
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_qconv.py -k "mixed or int8_resnet" > gpurun_out/r5/b14_qtests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b14_qtests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 600 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/b14_quant.log 2>&1 || exit 7
tail -1 gpurun_out/r5/b14_quant.log | head -c 4000
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
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b14_def_$i.log 2>&1 || exit 20
  ZOO_WGRAD256_MMAX=1048576 $T 200 python -u bench.py > gpurun_out/r5/b14_mmax_$i.log 2>&1 || exit 21
  ZOO_WGRAD256_MMAX=1048576 ZOO_WGRAD256_CMIN=64 $T 200 python -u bench.py > gpurun_out/r5/b14_cmin_$i.log 2>&1 || exit 22
done
for f in gpurun_out/r5/b14_{def,mmax,cmin}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
