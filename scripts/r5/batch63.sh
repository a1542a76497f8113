#!/bin/bash
# r5 batch 63: NCF regression check against the r4 wgrad settings
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 300 python -u bench.py --model ncf --batch 65536 --steps 100 --warmup 20 > gpurun_out/r5/b63_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_WG=1024 ZOO_WGRAD_DMA=0 $T 300 python -u bench.py --model ncf --batch 65536 --steps 100 --warmup 20 > gpurun_out/r5/b63_r4_$i.log 2>&1 || exit 11
done
for f in gpurun_out/r5/b63_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
