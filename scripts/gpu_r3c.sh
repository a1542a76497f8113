#!/bin/bash
# round-3 batch C: FRCNN / Keras-native / linear tests, ResNet A/B (igemm2 routing), BERT native vs hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_frcnn.py tests/test_gpu_keras_native.py tests/test_gpu_kernels.py tests/test_gpu_igemm2.py tests/test_gpu_native_nets.py -q --timeout 180 --timeout-method thread > gpurun_out/t_r3c.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r3c.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  ZOO_IGEMM2=0 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_c_off_$i.log 2>&1 || exit 5
  ZOO_IGEMM2=1 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_c_on_$i.log 2>&1 || exit 6
done
for f in gpurun_out/bench_c_*.log; do echo -n "$f "; grep -h '"metric"' $f | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['value'], d['ms_per_step'], d.get('final_loss'))"; done
for i in 1 2; do
  ZOO_LINEAR_BLAS=1 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_c_blas_$i.log 2>&1 || exit 7
  ZOO_LINEAR_BLAS=0 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_c_native_$i.log 2>&1 || exit 8
done
grep -h bench gpurun_out/bert_c_*.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/prof_bert_c.log 2>&1 || exit 9
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_bert -name "*.db" | head -1) 13 "BERT-base fine-tune b128 s128, native linears (13 steps traced)" > gpurun_out/prof_bert_c_summary.md 2>&1
head -30 gpurun_out/prof_bert_c_summary.md
