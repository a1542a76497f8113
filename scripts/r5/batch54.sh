#!/bin/bash
# r5 batch 54: HIP runtime settings A/B (kernel arguments in device memory)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 200 python -u bench.py > gpurun_out/r5/b54_def_$i.log 2>&1 || exit 10
  HIP_FORCE_DEV_KERNARG=1 $T 200 python -u bench.py > gpurun_out/r5/b54_kernarg_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b54_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"host_ms_per_step": [0-9.]*' $f)"; done
