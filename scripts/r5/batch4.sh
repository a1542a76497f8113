#!/bin/bash
# r5 batch 4: parity re-measure (+ fault), graph-captured BERT with in-backward optimizer (tests +
# A/B), NNEstimator input-path bench vs device-resident bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_ibo.py tests/test_gpu_graph_shapes.py -v --timeout 120 --timeout-method thread > gpurun_out/r5/b4_tests.log 2>&1
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5/b4_tests.log | tail -12
for i in 1 2; do
  $T 300 python -u bench.py --input featureset > gpurun_out/r5/b4_fs_$i.log 2>&1 || { tail -5 gpurun_out/r5/b4_fs_$i.log; exit 4; }
  $T 200 python -u bench.py > gpurun_out/r5/b4_dev_$i.log 2>&1 || exit 5
done
ZOO_COPY_STREAM=0 $T 300 python -u bench.py --input featureset > gpurun_out/r5/b4_fs_nocs.log 2>&1 || exit 6
for f in gpurun_out/r5/b4_{fs,dev}_*.log gpurun_out/r5/b4_fs_nocs.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
for g in "" "--graph"; do
  $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 $g > gpurun_out/r5/b4_bert$g.log 2>&1 || { tail -5 gpurun_out/r5/b4_bert$g.log; exit 7; }
  tail -1 gpurun_out/r5/b4_bert$g.log
done
$T 600 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity2 > gpurun_out/r5/parity2.log 2>&1 || { tail -20 gpurun_out/r5/parity2.log; exit 8; }
ZOO_FAULT_DGRAD=3:1.05 $T 300 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity2_fault vgg-16,mobilenet,inception-v1 > gpurun_out/r5/parity2_fault.log 2>&1 || { tail -20 gpurun_out/r5/parity2_fault.log; exit 9; }
echo parity-done
