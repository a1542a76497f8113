#!/bin/bash
# stem BN-ReLU-maxpool unrolled windows: numerics, kernel times, end to end (host time too)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/stem; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem_pool.py tests/test_gpu_resnet50_parity.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/st_rn -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit 3
DB=$(find /tmp/st_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 9 "stem" > $O/sum.md 2>&1
grep "maxpool" $O/sum.md
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/rn_$i.log 2>&1 || exit 4
  echo "resnet run=$i $(grep -o '"value": [0-9.]*' $O/rn_$i.log) $(grep -o '"host_ms_per_step": [0-9.]*' $O/rn_$i.log)"
done
