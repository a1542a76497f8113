#!/bin/bash
# rocprofv3 kernel trace of the ResNet-50 b256 bench step and the BERT-base step: per-kernel
# summary, one-step timeline and the critical-path attribution (tools/prof_step.py --critical)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
T="timeout -k 10"
TAG=${1:-r5}
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/r5/prof_rn_$TAG.log 2>&1 || exit 8
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 11 "ResNet-50 b256 training (bench.py under rocprofv3), $TAG" > gpurun_out/r5/prof_rn_${TAG}_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r5/prof_rn_${TAG}_step.md 2>&1
tail -45 gpurun_out/r5/prof_rn_${TAG}_step.md
if [ "$2" = "bert" ]; then
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 6 > gpurun_out/r5/prof_bert_$TAG.log 2>&1 || exit 9
DB=$(find /tmp/prof_bert -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r5/prof_bert_${TAG}_step.md 2>&1
tail -30 gpurun_out/r5/prof_bert_${TAG}_step.md
fi
