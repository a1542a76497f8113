#!/bin/bash
# round-3 batch F: fused NCF v2 (ILP layers, coalesced scatter, native prob-NLL), native-net parity
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_ncf_fused.py tests/test_jpeg.py tests/test_gpu_native_nets.py tests/test_gpu_zoo_kernels.py -v --timeout 300 --timeout-method thread > gpurun_out/t_r3f.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|logits rel" gpurun_out/t_r3f.log | tail -24
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
$T 300 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > gpurun_out/bench_ncf_f.log 2>&1 || exit 4
grep -h '"metric"' gpurun_out/bench_ncf_f.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ncf -o ncf -- python3 bench.py --model ncf --batch 65536 --steps 25 --warmup 5 > gpurun_out/prof_ncf_f.log 2>&1 || exit 8
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_ncf -name "*.db" | head -1) 32 "NCF ml-20m shape b65536, fused NCF kernels v2 (bench.py --model ncf under rocprofv3)" > gpurun_out/prof_ncf_f_summary.md 2>&1
head -24 gpurun_out/prof_ncf_f_summary.md
$T 400 python -u analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 20 > gpurun_out/mobilenet_train_f.log 2>&1 || exit 9
cat gpurun_out/mobilenet_train_f.log | tail -5
echo done
