#!/bin/bash
# round-3 batch G: GPU JPEG decode in serving -- tests, drain throughput A/B, open-loop latency
# curve, torchrun-launched one-worker-per-GPU path (1 GPU here)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_jpeg.py tests/test_serving.py tests/test_ncf_fused.py "tests/test_gpu_native_nets.py::test_backbone_matches_fp32_and_trains_natively" -k "not vgg and not alexnet and not densenet and not inception-v3" -v --timeout 180 --timeout-method thread > gpurun_out/t_r3g.log 2>&1
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
$T 300 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > gpurun_out/bench_ncf_g.log 2>&1 || exit 9
grep -h '"metric"' gpurun_out/bench_ncf_g.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_mbn -o mbn -- python3 analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 10 > gpurun_out/prof_mbn_g.log 2>&1 || exit 10
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_mbn -name "*.db" | head -1) 13 "MobileNet-v1 train b64 (zoo_models_bench.py under rocprofv3)" > gpurun_out/prof_mbn_g_summary.md 2>&1
head -40 gpurun_out/prof_mbn_g_summary.md
echo done
