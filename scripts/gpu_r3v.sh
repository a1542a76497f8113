#!/bin/bash
# round-3 batch V: 1x1 EPI 2 operand prefetch before the main loop (tests + same-box bench A/B + profile)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bn_mask or bn_backward_fusion or conv" tests/test_gpu_shortcut_bn.py > gpurun_out/t_r3v.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r3v.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ZOO_EPI2_BATCH=$v $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_v_${v}_$i.log 2>&1 || exit 2
    echo "epi2_batch=$v run $i: $(tail -1 gpurun_out/bench_v_${v}_$i.log | cut -c1-150)"
  done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_rn_v.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 8 "ResNet-50 b256 training (bench.py under rocprofv3), batched EPI 2 epilogue" > gpurun_out/prof_rn_v_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB > gpurun_out/prof_rn_v_step.md 2>&1
head -22 gpurun_out/prof_rn_v_summary.md
echo done
