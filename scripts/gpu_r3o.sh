#!/bin/bash
# round-3 batch O: Wide&Deep fused deep-input / head kernels (tests, bench, glue share)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sparse.py > gpurun_out/t_r3o.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/t_r3o.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
$T 300 python -u analytics-zoo_amd/tools/wnd_bench.py --batch 8192 --steps 30 --warmup 5 > gpurun_out/wnd_o_$i.log 2>&1 || exit 2
grep -v amdgpu.ids gpurun_out/wnd_o_$i.log | tail -1
done
$T 300 python -u analytics-zoo_amd/tools/glue_report.py --model wnd --rows 25 > gpurun_out/glue_o_wnd.md 2>&1 || exit 3
grep -v "amdgpu.ids\|Warn\|warn" gpurun_out/glue_o_wnd.md | cut -c1-250 | head -30
echo done
