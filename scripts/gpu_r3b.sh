#!/bin/bash
# round-3 batch B: new GPU tests, igemm2 bench (model-like epilogues), bench A/B igemm2 on/off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_keras_native.py tests/test_gpu_igemm2.py tests/test_gpu_ddp.py tests/test_gpu_round3.py -q --timeout 180 --timeout-method thread > gpurun_out/t_r3b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/t_r3b.log | grep -E "passed|failed|FAILED|Error" | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
$T 500 python -u analytics-zoo_amd/tools/igemm2_bench.py --tiles 0,1,5 --out gpurun_out/igemm2_bench_b.json > gpurun_out/igemm2_bench_b.log 2>&1 || exit 4
grep whole_network gpurun_out/igemm2_bench_b.log
for i in 1 2; do
  ZOO_IGEMM2=0 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_b_off_$i.log 2>&1 || exit 5
  ZOO_IGEMM2=1 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_b_on_$i.log 2>&1 || exit 6
done
for f in gpurun_out/bench_b_*.log; do echo -n "$f "; grep -h '"metric"' $f | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['value'], d['ms_per_step'], d['config']['grad_sync'], d.get('final_loss'), d.get('rccl_world'))"; done
