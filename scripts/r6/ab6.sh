#!/bin/bash
# r6 run 6: 256x192 auto-selection A/B on the BERT step (off / forward epilogues / all), isolated
# GEMMs with the auto choice, ConvLSTM3D kernel stats (fused vs per-step loop), default ResNet bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_igemm2.py tests/test_gpu_bert_parity.py -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ab6_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 300 python3 -u analytics-zoo_amd/tools/gemm_bench.py --bert > gpurun_out/r6/ab6_gemm_bert.log 2>&1 || exit 23
grep '"M"' gpurun_out/r6/ab6_gemm_bert.log | cut -c1-250
for i in 1 2; do
  for m in 0 1 2; do
    $T 300 python3 -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --i2-192 $m > gpurun_out/r6/ab6_bert_m${m}_$i.log 2>&1 || exit 31
    echo "m$m $(tail -1 gpurun_out/r6/ab6_bert_m${m}_$i.log | cut -c1-120)"
  done
done
for mode in fused loop; do
  rm -rf /tmp/prof_cl_$mode
  $T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_cl_$mode -o cl -- python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 16 --modes $mode --iters 3 > gpurun_out/r6/ab6_cl_$mode.log 2>&1 || exit 41
  f=$(find /tmp/prof_cl_$mode -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/r6/ab6_cl_${mode}_kernel_stats.csv
  head -16 "$f" | cut -d, -f1-4 | cut -c1-160
done
for i in 1 2; do
  $T 300 python -u bench.py > gpurun_out/r6/ab6_default_$i.log 2>&1 || exit 22
  tail -1 gpurun_out/r6/ab6_default_$i.log | cut -c1-200
done
