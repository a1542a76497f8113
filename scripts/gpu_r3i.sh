#!/bin/bash
# round-3 batch I: GELU-backward dgrad routed to igemm2, LDS-tiled 1x1 weight flip (BERT A/B +
# profile), current ResNet-50 bench + profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_gelu_dgrad.py tests/test_gpu_kernels.py tests/test_gpu_residual_grad.py tests/test_gpu_keras_th.py -v --timeout 300 --timeout-method thread > gpurun_out/t_r3i.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t_r3i.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  ZOO_GELU_DGRAD=1 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_i_fused_$i.log 2>&1 || exit 4
  ZOO_GELU_DGRAD=0 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_i_sep_$i.log 2>&1 || exit 5
done
grep -h '"bench"' gpurun_out/bert_i_*.log
$T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_resnet_i.log 2>&1 || exit 6
grep -h '"metric"' gpurun_out/bench_resnet_i.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/prof_bert_i.log 2>&1 || exit 11
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_bert -name "*.db" | head -1) 13 "BERT-base fine-tune b128 s128, native linears, GELU backward in the igemm2 dgrad epilogue, tiled weight flip (bert_train.py under rocprofv3)" > gpurun_out/prof_bert_i_summary.md 2>&1
head -24 gpurun_out/prof_bert_i_summary.md
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_rn_i.log 2>&1 || exit 12
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_rn -name "*.db" | head -1) 8 "ResNet-50 b256 training, round 3 (bench.py --steps 5 --warmup 3 under rocprofv3; 8 steps traced)" > gpurun_out/prof_rn_i_summary.md 2>&1
head -40 gpurun_out/prof_rn_i_summary.md
echo done
