#!/bin/bash
# round-3 batch A: new GPU tests, bench A/B igemm2 on/off, then the PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_round3.py -x -q --timeout 180 --timeout-method thread > gpurun_out/t_r3a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t_r3a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  ZOO_IGEMM2=0 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_i2off_$i.log 2>&1 || exit 5
  ZOO_IGEMM2=1 $T 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_i2on_$i.log 2>&1 || exit 6
done
grep -h '"metric"' gpurun_out/bench_i2*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['value'], d['ms_per_step'], d['config']['grad_sync'], d.get('final_loss'))"
bash scripts/gpu_pmc_igemm2.sh
