#!/bin/bash
# MFMA probe (fixed), ConvLSTM sequence path tests + bench, NCF loss tests + bench + profile
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/misc
timeout -k 5 60 ./analytics-zoo_amd/tools/mfma_probe > gpurun_out/misc/probe2.log 2>&1; cat gpurun_out/misc/probe2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad256.py tests/test_gpu_drop_ln.py tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py tests/test_ncf_fused.py -x -q -k "convlstm or ConvLSTM or prob_nll or ncf or wgrad or fused or bert_block" --timeout 120 --timeout-method thread > gpurun_out/misc/b_tests.log 2>&1
echo "tests rc=$?"; tail -4 gpurun_out/misc/b_tests.log
timeout -k 10 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/misc/convlstm_bench.log 2>&1
echo "convlstm bench rc=$?"; tail -2 gpurun_out/misc/convlstm_bench.log
timeout -k 10 200 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > gpurun_out/misc/bench_ncf.log 2>&1
echo "ncf bench rc=$?"; tail -1 gpurun_out/misc/bench_ncf.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ncf -o ncf -- python3 bench.py --model ncf --batch 65536 --steps 32 --warmup 10 > gpurun_out/misc/prof_ncf.log 2>&1 || exit 9
DB=$(find /tmp/prof_ncf -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 42 "NCF ml-20m shape b65536 (bench.py --model ncf under rocprofv3), round 4" > gpurun_out/misc/ncf_prof.md 2>&1
head -24 gpurun_out/misc/ncf_prof.md
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/misc/bench_rn_$i.log 2>&1 || exit 10
  echo "resnet run=$i $(grep -o '"value": [0-9.]*' gpurun_out/misc/bench_rn_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/misc/bench_rn_$i.log)"
done
timeout -k 10 240 python -u analytics-zoo_amd/tools/conv_sweep.py --detail --roofline gpurun_out/misc/resnet50_roofline.md > gpurun_out/misc/conv_sweep.log 2>&1 || exit 11
tail -1 gpurun_out/misc/conv_sweep.log
bash scripts/r4/prof_resnet.sh c3 > gpurun_out/misc/prof_rn_c3.out 2>&1 || exit 12
head -30 gpurun_out/prof_rn_c3_summary.md
