#!/bin/bash
# per-shape conv time of ResNet-50 b256 under each forced igemm2 tile (0 = default routing)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for t in 0 1 4 6 7; do
  ZOO_IGEMM2_TILE=$t timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops fwd,dgrad --detail > gpurun_out/sweep_t$t.log 2>&1 || exit 1
  tail -1 gpurun_out/sweep_t$t.log
done
