#!/bin/bash
# round-3 batch J: glue attribution for W&D / SSD / NCF steps, serving GPU test
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_kernels.py -k serving -v --timeout 200 --timeout-method thread > gpurun_out/t_r3j.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t_r3j.log | tail -4
for m in wnd ssd ncf; do
  $T 300 python -u analytics-zoo_amd/tools/glue_report.py --model $m > gpurun_out/glue_$m.md 2>&1 || exit 3
  grep -v amdgpu.ids gpurun_out/glue_$m.md | head -24
done
echo done
