#!/bin/bash
# r5 batch 16: native comm tests; ConvLSTM with batched weight staging (tests, bench, profile);
# wgrad256 routing for the 802816-row 1x1 weight gradients (3 runs each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm_native.py tests/test_gpu_ddp.py \
  tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py -k "comm or ddp or forced or zero1 or zombie or wire or ConvLSTM or convlstm" > gpurun_out/r5/b16_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r5/b16_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b16_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b16_convlstm_bench.log
$T 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cl -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --iters 3 > gpurun_out/r5/b16_prof_cl.log 2>&1 || exit 12
DB=$(find /tmp/prof_cl -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM2D T=32 bench (3 modes, 5 iters each)" > gpurun_out/r5/b16_prof_cl_summary.md 2>&1
grep -E "convlstm|lstm_step|elementwise|Fill|copy" gpurun_out/r5/b16_prof_cl_summary.md | head -14
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b16_def_$i.log 2>&1 || exit 20
  ZOO_WGRAD256_MMAX=1048576 $T 200 python -u bench.py > gpurun_out/r5/b16_mmax_$i.log 2>&1 || exit 21
done
for f in gpurun_out/r5/b16_{def,mmax}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
