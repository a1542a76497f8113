#!/bin/bash
# round-3 batch Z: shortcut-first backward at stage transitions (tests + bench A/B + profile), BERT profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "resnet or shortcut" tests/test_gpu_shortcut_bn.py tests/test_gpu_resnet50_parity.py tests/test_gpu_native_nets.py > gpurun_out/t_r3z.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3z.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ZOO_SHORTCUT_FIRST=$v $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_z_${v}_$i.log 2>&1 || exit 2
    echo "shortcut_first=$v run $i: $(tail -1 gpurun_out/bench_z_${v}_$i.log | cut -c1-150)"
  done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_rn_z.log 2>&1 || exit 4
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 $GRAFT_REPO_ROOT/analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert_z.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 8 "ResNet-50 b256 training (bench.py under rocprofv3), round-3 final: batched backward epilogues, shortcut-first stage transitions" > gpurun_out/prof_rn_z_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB > gpurun_out/prof_rn_z_step.md 2>&1
DB2=$(find /tmp/prof_bert -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB2 13 "BERT-base fine-tune b128 s128 (bert_train.py under rocprofv3), round-3 final: LayerNorm residual-gradient add, act_colsum 256 blocks" > gpurun_out/prof_bert_z_summary.md 2>&1
head -12 gpurun_out/prof_rn_z_summary.md; head -30 gpurun_out/prof_bert_z_summary.md
echo done
