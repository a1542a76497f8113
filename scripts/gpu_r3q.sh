#!/bin/bash
# round-3 batch Q: ResNet-50 glue attribution; wgrad256 split-count A/B on the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u analytics-zoo_amd/tools/glue_report.py --model resnet --rows 30 --steps 2 > gpurun_out/glue_q_resnet.md 2>&1 || exit 1
grep -v "amdgpu.ids\|Warn\|warn" gpurun_out/glue_q_resnet.md | cut -c1-260 | head -36
for wg in 256 512 128; do
  ZOO_WGRAD256_WG=$wg $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_q_$wg.log 2>&1 || exit 2
  echo "wg=$wg: $(grep '"metric"' gpurun_out/bench_q_$wg.log | cut -c1-110)"
done
echo done
