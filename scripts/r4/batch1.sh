#!/bin/bash
# round-4 validation batch 1: MFMA probe, new-kernel numerics, c3 read-schedule A/B, ResNet /
# BERT end-to-end, ConvLSTM sequence bench
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/b1; mkdir -p $O
timeout -k 5 60 ./analytics-zoo_amd/tools/mfma_probe > $O/probe.log 2>&1; cat $O/probe.log
timeout -k 10 420 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_wgrad256.py tests/test_gpu_drop_ln.py \
  tests/test_gpu_convlstm_seq.py tests/test_ncf_fused.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit 2
S=analytics-zoo_amd/tools/igemm2_one.py
kt() {
  n=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/c3p/$n -o k -- python3 $S "$@" > $O/${n}.log 2>&1 || return 1
  f=$(find /tmp/c3p/$n -name "*.db" | head -1)
  echo "$n $(python3 analytics-zoo_amd/tools/prof_summary.py $f 20 x | grep -m1 'c3_kernel')"
}
for late in 0 1; do
  ZOO_C3_LATE=$late kt fwd_late$late --conv 56,64,64,3,1,1 || exit 3
  ZOO_C3_LATE=$late kt dgrad_late$late --conv 56,64,64,3,1,1 --dgrad || exit 3
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_rn_$i.log 2>&1 || exit 4
  echo "resnet run=$i $(grep -o '"value": [0-9.]*' $O/bench_rn_$i.log) $(grep -o '"final_loss": [0-9.]*' $O/bench_rn_$i.log)"
done
for f in 1 0; do
  ZOO_DROP_LN_FUSE=$f timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/bert_dln$f.log 2>&1 || exit 5
  echo "DROP_LN_FUSE=$f $(tail -1 $O/bert_dln$f.log)"
done
timeout -k 10 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > $O/convlstm_bench.log 2>&1 || exit 6
tail -3 $O/convlstm_bench.log
