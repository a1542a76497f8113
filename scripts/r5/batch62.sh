#!/bin/bash
# r5 batch 62: NCF (ml-20m shape, b65536) and the featureset input-path bench on the final tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > gpurun_out/r5/b62_ncf.log 2>&1 || exit 10
grep '"metric"' gpurun_out/r5/b62_ncf.log | cut -c1-260
$T 300 python -u bench.py --input featureset > gpurun_out/r5/b62_featureset.log 2>&1 || exit 11
grep '"metric"' gpurun_out/r5/b62_featureset.log | cut -c1-200
