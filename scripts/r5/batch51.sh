#!/bin/bash
# r5 batch 51: tiled-wgrad workgroup target around 512 (with DMA staging) and the partial-buffer threshold
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b51_def_$i.log 2>&1 || exit 10
  ZOO_WGRAD_WG=448 $T 200 python -u bench.py > gpurun_out/r5/b51_wg448_$i.log 2>&1 || exit 11
  ZOO_WGRAD_WG=640 $T 200 python -u bench.py > gpurun_out/r5/b51_wg640_$i.log 2>&1 || exit 12
  ZOO_WGRAD_PARTIAL_MB=8 $T 200 python -u bench.py > gpurun_out/r5/b51_pmb8_$i.log 2>&1 || exit 13
  ZOO_WGRAD_PARTIAL_MB=64 $T 200 python -u bench.py > gpurun_out/r5/b51_pmb64_$i.log 2>&1 || exit 14
done
for f in gpurun_out/r5/b51_*_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
