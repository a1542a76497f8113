#!/bin/bash
# round-3 batch S (re-entry): BN ReLU-mask modes + 4-row BN backward apply (tests + same-box bench A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bn_mask or bn_backward_fusion or shortcut" tests/test_gpu_shortcut_bn.py > gpurun_out/t_r3s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t_r3s.log; [ $rc = 0 ] || exit 1
for r in 2 4; do
  ZOO_BN_BWD_ROWS=$r $T 300 python -u analytics-zoo_amd/tools/bn_bench.py > gpurun_out/bn_bench_s_$r.log 2>&1 || exit 3
  echo "bwd rows $r:"; grep -v amdgpu.ids gpurun_out/bn_bench_s_$r.log
done
for i in 1 2; do
  for v in "0 2" "1 2" "1 4"; do
    set -- $v
    ZOO_BN_MASK=$1 ZOO_BN_BWD_ROWS=$2 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_s_$1_$2_$i.log 2>&1 || exit 2
    echo "bn_mask=$1 bwd_rows=$2 run $i: $(tail -1 gpurun_out/bench_s_$1_$2_$i.log | cut -c1-150)"
  done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_rn_s.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 8 "ResNet-50 b256 training (bench.py under rocprofv3), BN mask modes + 4-row BN backward apply" > gpurun_out/prof_rn_s_summary.md 2>&1
python3 analytics-zoo_amd/tools/prof_step.py $DB > gpurun_out/prof_rn_s_step.md 2>&1
head -25 gpurun_out/prof_rn_s_summary.md
for i in 1 2; do
  for v in "1024 256" "256 256" "1024 128"; do
    set -- $v
    ZOO_COLSUM_BLOCKS=$1 ZOO_WGRAD256_WG=$2 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_s_$1_$2_$i.log 2>&1 || exit 5
    echo "bert colsum_blocks=$1 wgrad256_wg=$2 run $i: $(grep -v amdgpu.ids gpurun_out/bert_s_$1_$2_$i.log | tail -1 | cut -c1-160)"
  done
done
echo done
