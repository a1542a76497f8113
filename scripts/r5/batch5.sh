#!/bin/bash
# r5 batch 5: parity with emulated bf16 storage (+ fault), quant tests + quant bench (per-channel int8),
# dropout-under-graph test, BERT graph replay host cost
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_qconv.py tests/test_gpu_ibo.py -v --timeout 120 --timeout-method thread > gpurun_out/r5/b5_tests.log 2>&1
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5/b5_tests.log | tail -16
$T 600 python -u analytics-zoo_amd/tools/quant_bench.py --no-dynamic > gpurun_out/r5/quant_bench_r5.log 2>&1 || { tail -5 gpurun_out/r5/quant_bench_r5.log; exit 3; }
tail -1 gpurun_out/r5/quant_bench_r5.log
$T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --graph > gpurun_out/r5/b5_bert_graph.log 2>&1 || exit 4
tail -1 gpurun_out/r5/b5_bert_graph.log
$T 600 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity3 > gpurun_out/r5/parity3.log 2>&1 || { tail -20 gpurun_out/r5/parity3.log; exit 8; }
ZOO_FAULT_DGRAD=3:1.05 $T 300 python -u analytics-zoo_amd/tools/parity_dump.py gpurun_out/r5/parity3_fault vgg-16,mobilenet,inception-v1,densenet-161 > gpurun_out/r5/parity3_fault.log 2>&1 || { tail -20 gpurun_out/r5/parity3_fault.log; exit 9; }
echo parity-done
