#!/bin/bash
# r5 batch 49: BERT-base b128 critical-path profile on the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 6 > gpurun_out/r5/b49_prof_bert.log 2>&1 || exit 9
DB=$(find /tmp/prof_bert -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r5/b49_bert_step.md 2>&1
python3 analytics-zoo_amd/tools/prof_summary.py $DB 5 "BERT-base b128 s128 training, r5" > gpurun_out/r5/b49_bert_summary.md 2>&1
tail -40 gpurun_out/r5/b49_bert_step.md
