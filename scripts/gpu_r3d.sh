#!/bin/bash
# round-3 batch D: ROI / FRCNN fixes, per-layer parity of the failing native nets, linear epilogue cost
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_frcnn.py -q --timeout 120 --timeout-method thread > gpurun_out/t_r3d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t_r3d.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
$T 300 python -u analytics-zoo_amd/tools/linear_epi_bench.py > gpurun_out/linear_epi.log 2>&1 || exit 4
cat gpurun_out/linear_epi.log
for n in mobilenet inception-v3 densenet-161 inception-v1; do
  hw=224; [ $n = inception-v3 ] && hw=299
  $T 300 python -u analytics-zoo_amd/tools/layer_parity.py --net $n --hw $hw --out gpurun_out/parity_$n.json > gpurun_out/parity_$n.log 2>&1 || exit 5
done
echo done
