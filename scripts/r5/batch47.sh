#!/bin/bash
# r5 batch 47: igemm tile width / staging re-check on the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b47_def_$i.log 2>&1 || exit 10
  ZOO_IGEMM_BN=128 $T 200 python -u bench.py > gpurun_out/r5/b47_bn128_$i.log 2>&1 || exit 11
  ZOO_IGEMM_DMA=0 $T 200 python -u bench.py > gpurun_out/r5/b47_nodma_$i.log 2>&1 || exit 12
  ZOO_C3_LATE=1 $T 200 python -u bench.py > gpurun_out/r5/b47_c3late_$i.log 2>&1 || exit 13
done
for f in gpurun_out/r5/b47_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
