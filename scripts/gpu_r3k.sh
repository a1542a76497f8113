#!/bin/bash
# round-3 batch K: W&D bf16 deep tower (bench + glue), SSD glue attribution
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u analytics-zoo_amd/tools/wnd_bench.py --batch 8192 --steps 30 --warmup 5 > gpurun_out/wnd_k.log 2>&1 || exit 2
grep -v amdgpu.ids gpurun_out/wnd_k.log | tail -2
for m in wnd ssd; do
  $T 300 python -u analytics-zoo_amd/tools/glue_report.py --model $m --rows 25 > gpurun_out/glue_k_$m.md 2>&1 || exit 3
  grep -v "amdgpu.ids\|Warn\|warn" gpurun_out/glue_k_$m.md | head -30
done
echo done
