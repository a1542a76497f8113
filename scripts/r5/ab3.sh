#!/bin/bash
# r5 batch 3: new GPU tests (wgrad256 atomic split-K, lowering: grouped / depthwise / deconv / GRU /
# MTNet, hipGraph over three shapes, lowered-conv cache), the atomic split-K A/B, per-layer parity dump
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_wgrad256.py tests/test_gpu_native_import.py tests/test_gpu_graph_shapes.py tests/test_gpu_ibo.py -v --timeout 120 --timeout-method thread > gpurun_out/r5/ab3_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5/ab3_tests.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
for i in 1 2; do
  ZOO_WGRAD256_ATOMIC_MB=0 $T 200 python -u bench.py > gpurun_out/r5/ab2_off_$i.log 2>&1 || exit 4
  $T 200 python -u bench.py > gpurun_out/r5/ab2_def_$i.log 2>&1 || exit 5
  ZOO_WGRAD256_ATOMIC_MB=100000 ZOO_WGRAD_PARTIAL_MB=0 $T 200 python -u bench.py > gpurun_out/r5/ab2_all_$i.log 2>&1 || exit 6
done
for f in gpurun_out/r5/ab2_{off,def,all}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
$T 600 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity > gpurun_out/r5/parity_dump.log 2>&1 || { tail -20 gpurun_out/r5/parity_dump.log; exit 7; }
tail -3 gpurun_out/r5/parity_dump.log
