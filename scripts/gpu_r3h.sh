#!/bin/bash
# round-3 batch H: GELU-backward-in-dgrad (BERT A/B), sliding-window depthwise wgrad (MobileNet),
# cached-table JPEG decode (serving, natural + noise images), W&D / SSD profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_gelu_dgrad.py tests/test_gpu_zoo_kernels.py tests/test_gpu_pointwise.py tests/test_gpu_residual_grad.py tests/test_ncf_fused.py tests/test_jpeg.py tests/test_gpu_qconv.py -v --timeout 300 --timeout-method thread > gpurun_out/t_r3h.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t_r3h.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
$T 300 python -u analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 20 > gpurun_out/mobilenet_train_h.log 2>&1 || exit 3
$T 300 python -u analytics-zoo_amd/tools/quant_bench.py --batch 256 --iters 20 --no-dynamic > gpurun_out/quant_h.log 2>&1 || exit 31
grep -h '"bench"' gpurun_out/quant_h.log
grep -h '"model"' gpurun_out/mobilenet_train_h.log
for i in 1 2; do
  ZOO_GELU_DGRAD=1 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_h_fused_$i.log 2>&1 || exit 4
  ZOO_GELU_DGRAD=0 $T 300 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_h_sep_$i.log 2>&1 || exit 5
done
tail -n 2 gpurun_out/bert_h_*.log
$T 400 python -u analytics-zoo_amd/tools/serving_bench.py e2e --drain --batch 128 --images 4096 --images-kind natural > gpurun_out/srv_h_drain_natural.log 2>&1 || exit 6
$T 400 python -u analytics-zoo_amd/tools/serving_bench.py e2e --drain --batch 128 --images 4096 --images-kind noise > gpurun_out/srv_h_drain_noise.log 2>&1 || exit 7
grep -h '"bench"' gpurun_out/srv_h_drain_*.log
$T 400 python -u analytics-zoo_amd/tools/serving_bench.py e2e --batch 128 --images 8192 --client-procs 6 --images-kind natural > gpurun_out/srv_h_e2e_natural.log 2>&1 || exit 8
grep -h '"bench"' gpurun_out/srv_h_e2e_natural.log
$T 600 python -u analytics-zoo_amd/tools/serving_bench.py openloop --batch 128 --duration 6 --images-kind natural > gpurun_out/srv_h_openloop.log 2>&1 || exit 9
grep -h '"bench"' gpurun_out/srv_h_openloop.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mbn -o mbn -- python3 analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode train --batch 64 --steps 10 > gpurun_out/prof_mbn_h.log 2>&1 || exit 10
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_mbn -name "*.db" | head -1) 13 "MobileNet-v1 train b64, sliding-window depthwise wgrad (zoo_models_bench.py under rocprofv3)" > gpurun_out/prof_mbn_h_summary.md 2>&1
head -16 gpurun_out/prof_mbn_h_summary.md
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/prof_bert_h.log 2>&1 || exit 11
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_bert -name "*.db" | head -1) 13 "BERT-base fine-tune b128 s128, native linears + fused GELU backward (bert_train.py under rocprofv3)" > gpurun_out/prof_bert_h_summary.md 2>&1
head -24 gpurun_out/prof_bert_h_summary.md
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_wnd -o wnd -- python3 analytics-zoo_amd/tools/wnd_bench.py --batch 8192 --steps 20 --warmup 5 > gpurun_out/prof_wnd_h.log 2>&1 || exit 12
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_wnd -name "*.db" | head -1) 25 "Wide&Deep b8192 train (wnd_bench.py under rocprofv3)" > gpurun_out/prof_wnd_h_summary.md 2>&1
head -24 gpurun_out/prof_wnd_h_summary.md
$T 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ssd -o ssd -- python3 analytics-zoo_amd/tools/zoo_models_bench.py --models ssd300 --mode train --batch 16 --steps 10 > gpurun_out/prof_ssd_h.log 2>&1 || exit 13
python3 analytics-zoo_amd/tools/prof_summary.py $(find /tmp/prof_ssd -name "*.db" | head -1) 13 "SSD-300 VGG train b16 (zoo_models_bench.py under rocprofv3)" > gpurun_out/prof_ssd_h_summary.md 2>&1
head -24 gpurun_out/prof_ssd_h_summary.md
echo done
