#!/bin/bash
# r6 first GPU check: full GPU suite, featureset (default) vs device bench pair, BERT eager vs
# graph step traces with the critical-path attribution
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/gpu_tests_first.log 2>&1
rc=$?
tail -5 gpurun_out/r6/gpu_tests_first.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 300 python -u bench.py > gpurun_out/r6/bench_fs_$i.log 2>&1 || exit 21
  tail -1 gpurun_out/r6/bench_fs_$i.log
  $T 300 python -u bench.py --input device > gpurun_out/r6/bench_dev_$i.log 2>&1 || exit 22
  tail -1 gpurun_out/r6/bench_dev_$i.log
done
for mode in eager graph; do
  flag=""; [ $mode = graph ] && flag="--graph"
  $T 300 python3 -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 $flag > gpurun_out/r6/bert_$mode.log 2>&1 || exit 30
  tail -1 gpurun_out/r6/bert_$mode.log
  rm -rf /tmp/prof_bert_$mode
  $T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert_$mode -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 6 $flag > gpurun_out/r6/prof_bert_$mode.log 2>&1 || exit 31
  DB=$(find /tmp/prof_bert_$mode -name "*.db" | head -1)
  python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r6/prof_bert_${mode}_step.md 2>&1
  tail -25 gpurun_out/r6/prof_bert_${mode}_step.md
done
