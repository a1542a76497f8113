#!/bin/bash
# per-layer parity with bf16-rounded twin weights, then the same with a 5 % fault in one conv dgrad
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity2 > gpurun_out/r5/parity2.log 2>&1 || { tail -20 gpurun_out/r5/parity2.log; exit 7; }
ZOO_FAULT_DGRAD=3:1.05 $T 300 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity2_fault vgg-16,mobilenet,inception-v1 > gpurun_out/r5/parity2_fault.log 2>&1 || { tail -20 gpurun_out/r5/parity2_fault.log; exit 8; }
tail -3 gpurun_out/r5/parity2_fault.log
