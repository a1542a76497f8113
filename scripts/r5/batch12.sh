#!/bin/bash
# r5 batch 12: prologue restricted to 64-channel units (tests + same-box A/B), faster apply
# fallback; ConvLSTM step kernels with LDS-staged weights (tests + bench + kernel profile)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfold.py tests/test_gpu_convlstm_seq.py \
  tests/test_gpu_keras_native.py -k "bnfold or prologue or ConvLSTM or convlstm" > gpurun_out/r5/b12_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r5/b12_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b12_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b12_convlstm_bench.log
for i in 1 2; do
  ZOO_BN_FOLD=1 $T 200 python -u bench.py > gpurun_out/r5/b12_pro_$i.log 2>&1 || exit 10
  ZOO_BN_FOLD=0 $T 200 python -u bench.py > gpurun_out/r5/b12_nopro_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b12_{pro,nopro}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
$T 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cl -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --iters 3 > gpurun_out/r5/b12_prof_cl.log 2>&1 || exit 12
DB=$(find /tmp/prof_cl -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM2D T=32 bench (3 modes, 5 iters each)" > gpurun_out/r5/b12_prof_cl_summary.md 2>&1
head -30 gpurun_out/r5/b12_prof_cl_summary.md
