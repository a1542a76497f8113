#!/bin/bash
# round-3 batch G: GPU JPEG decode in serving -- tests, drain throughput A/B, open-loop latency
# curve, torchrun-launched one-worker-per-GPU path (1 GPU here)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_jpeg.py tests/test_serving.py -v --timeout 180 --timeout-method thread > gpurun_out/t_r3g.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t_r3g.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
$T 400 python -u analytics-zoo_amd/tools/serving_bench.py e2e --drain --batch 128 --images 4096 > gpurun_out/srv_drain_gpujpeg.log 2>&1 || exit 4
ZOO_SERVING_GPU_JPEG=0 $T 400 python -u analytics-zoo_amd/tools/serving_bench.py e2e --drain --batch 128 --images 4096 > gpurun_out/srv_drain_cpu.log 2>&1 || exit 5
grep -h '"bench"' gpurun_out/srv_drain_*.log
$T 400 python -u analytics-zoo_amd/tools/serving_bench.py e2e --batch 128 --images 8192 --client-procs 6 > gpurun_out/srv_e2e_gpujpeg.log 2>&1 || exit 6
grep -h '"bench"' gpurun_out/srv_e2e_gpujpeg.log
$T 600 python -u analytics-zoo_amd/tools/serving_bench.py openloop --batch 128 --duration 6 > gpurun_out/srv_openloop.log 2>&1 || exit 7
grep -h '"bench"' gpurun_out/srv_openloop.log
$T 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 analytics-zoo_amd/tools/serving_bench.py dist --batch 128 --images 4096 > gpurun_out/srv_dist1.log 2>&1 || exit 8
grep -h '"bench"' gpurun_out/srv_dist1.log
echo done
