#!/bin/bash
# kernel-trace profiles of the current ResNet-50 and BERT-base steps (side stream + in-backward optimizer on)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pb; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pb_rn -o rn -- python3 bench.py --steps 8 --warmup 3 > $O/rn.log 2>&1 || exit 2
DB=$(find /tmp/pb_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 11 "ResNet-50 b256 training (bench.py under rocprofv3), round 4: side stream + in-backward optimizer" > $O/rn_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB > $O/rn_step.md 2>&1
head -14 $O/rn_summary.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pb_bert -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > $O/bert.log 2>&1 || exit 3
DB=$(find /tmp/pb_bert -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 13 "BERT-base fine-tune b128 s128 (bert_train.py under rocprofv3), round 4" > $O/bert_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB "softmax_xent_kernel" > $O/bert_step.md 2>&1
head -30 $O/bert_summary.md
