#!/bin/bash
# round-3 batch R: LayerNorm backward v2 (tests, BERT A/B, kernel profile)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm" > gpurun_out/t_r3r.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3r.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ZOO_LN_BWD_V2=$v $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_r_${v}_$i.log 2>&1 || exit 2
    echo "ln_v2=$v run $i: $(grep -v amdgpu.ids gpurun_out/bert_r_${v}_$i.log | tail -1 | cut -c1-200)"
  done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 $GRAFT_REPO_ROOT/analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert_r.log 2>&1 || exit 3
cd $GRAFT_REPO_ROOT
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_bert -name "*.db" | head -1) 13 "BERT-base fine-tune b128 s128 (bert_train.py under rocprofv3)" > gpurun_out/prof_bert_r_summary.md 2>&1
head -30 gpurun_out/prof_bert_r_summary.md
$T 300 python -u analytics-zoo_amd/tools/glue_report.py --model bert --rows 25 --steps 2 > gpurun_out/glue_r_bert.md 2>&1 || exit 4
grep -v "amdgpu.ids\\|Warn\\|warn" gpurun_out/glue_r_bert.md | cut -c1-200 | head -30
echo done
