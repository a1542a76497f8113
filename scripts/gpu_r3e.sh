#!/bin/bash
# round-3 batch E: fused NCF kernels (tests, bench A/B, rocprof), lean linear epilogue, BN probe
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_ncf_fused.py tests/test_frcnn.py -x -v --timeout 180 --timeout-method thread > gpurun_out/t_r3e.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r3e.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
$T 300 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > gpurun_out/bench_ncf_fused.log 2>&1 || exit 4
ZOO_NCF_FUSED=0 $T 300 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > gpurun_out/bench_ncf_layers.log 2>&1 || exit 5
grep -h '"metric"' gpurun_out/bench_ncf_*.log
$T 300 python -u analytics-zoo_amd/tools/linear_epi_bench.py > gpurun_out/linear_epi_e.log 2>&1 || exit 6
cat gpurun_out/linear_epi_e.log
$T 300 python -u analytics-zoo_amd/tools/bn_probe.py > gpurun_out/bn_probe.log 2>&1 || exit 7
cat gpurun_out/bn_probe.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ncf -o ncf -- python3 bench.py --model ncf --batch 65536 --steps 25 --warmup 5 > gpurun_out/prof_ncf_e.log 2>&1 || exit 8
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_ncf -name "*.db" | head -1) 32 "NCF ml-20m shape b65536, fused NCF kernels (bench.py --model ncf under rocprofv3)" > gpurun_out/prof_ncf_e_summary.md 2>&1
head -24 gpurun_out/prof_ncf_e_summary.md
for i in 1 2; do
  ZOO_LINEAR_BLAS=0 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_e_native_$i.log 2>&1 || exit 9
  ZOO_LINEAR_BLAS=1 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_e_blas_$i.log 2>&1 || exit 10
done
grep -h bench gpurun_out/bert_e_*.log
echo done
