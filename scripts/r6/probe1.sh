#!/bin/bash
# gconv numerics with full failure output; RCCL collective capture probe, one collective per process
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_kernels.py -k "grouped_conv_kernels" -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r6/probe1_gconv.log 2>&1
rc=$?; tail -3 gpurun_out/r6/probe1_gconv.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
# stop at the first crash (segfault / abort / timeout): nothing more runs on the GPU after it
for op in all_reduce all_gather all_to_all reduce_scatter; do
  $T 120 python3 -u analytics-zoo_amd/tools/probe_comm_capture.py $op > gpurun_out/r6/probe1_$op.log 2>&1
  rc=$?; echo "$op rc=$rc"; tail -2 gpurun_out/r6/probe1_$op.log
  [ $rc -eq 0 ] || exit $rc
done
