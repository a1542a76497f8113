#!/bin/bash
# round-3 batch L: SSD native NormalizeScale + hard-negative mining (tests, step time, glue share)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bmm.py -k "ssd or normalize" > gpurun_out/t_r3l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/t_r3l.log; [ $rc = 0 ] || exit 1
$T 300 python -u analytics-zoo_amd/tools/zoo_models_bench.py --models ssd300 --mode train --batch 16 --steps 20 > gpurun_out/ssd_l.log 2>&1 || exit 2
grep -v amdgpu.ids gpurun_out/ssd_l.log | tail -3
$T 300 python -u analytics-zoo_amd/tools/glue_report.py --model ssd --rows 25 > gpurun_out/glue_l_ssd.md 2>&1 || exit 3
grep -v "amdgpu.ids\|Warn\|warn" gpurun_out/glue_l_ssd.md | head -34
echo done
