#!/bin/bash
# r6 A/B 1: band weight gradient (ZOO_WGRAD_BAND), flip prefetch (ZOO_FLIP_PREFETCH), BN-backward
# prologue on the 256-wide stage-1 units (ZOO_BN_FOLD_K=64,256); grouped conv tests; ResNet and
# BERT step traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_native_import.py tests/test_gpu_kernels.py tests/test_gpu_comm_native.py \
  -k "wgrad or group or grouped_conv" -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/ab1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab1_tests.log
# test failures (1) do not stop the A/B; a crash, fault or timeout does
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" $T 300 python -u bench.py --input device > gpurun_out/r6/ab1_$tag.log 2>&1 || exit 21
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6/ab1_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
}
for i in 1 2; do
  run base$i ZOO_WGRAD_BAND=0 ZOO_FLIP_PREFETCH=0
  run band$i ZOO_WGRAD_BAND=1 ZOO_FLIP_PREFETCH=0
  run bandflip$i ZOO_WGRAD_BAND=1 ZOO_FLIP_PREFETCH=1
  run bandflipfold$i ZOO_WGRAD_BAND=1 ZOO_FLIP_PREFETCH=1 ZOO_BN_FOLD_K=64,256
done
rm -rf /tmp/prof_rn
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 bench.py --input device --steps 8 --warmup 3 > gpurun_out/r6/prof_rn_ab1.log 2>&1 || exit 8
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r6/prof_rn_ab1_step.md 2>&1
tail -40 gpurun_out/r6/prof_rn_ab1_step.md
for mode in eager graph; do
  # loss kernel as the boundary: one per step; 3 warm-up + 10 timed + 5 idle-device probe steps
  # (+ 5 bare replays with --graph): the period picked lies inside the pipelined timed loop
  flag=""; back=8; [ $mode = graph ] && flag="--graph" && back=13
  rm -rf /tmp/prof_bert_$mode
  $T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert_$mode -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 $flag > gpurun_out/r6/prof_bert_$mode.log 2>&1 || exit 31
  DB=$(find /tmp/prof_bert_$mode -name "*.db" | head -1)
  python3 analytics-zoo_amd/tools/prof_step.py $DB softmax_xent $back --critical > gpurun_out/r6/prof_bert_${mode}_step.md 2>&1
  tail -30 gpurun_out/r6/prof_bert_${mode}_step.md
done
# last: the whole-step hipGraph over the native comm layer (a crash here ends the call)
$T 300 python -u -m pytest tests/test_gpu_comm_native.py -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/ab1_fullstep.log 2>&1
echo "fullstep rc=$?"; tail -3 gpurun_out/r6/ab1_fullstep.log
