#!/bin/bash
# r5 batch 26: stem max-pool backward over 2x2 quads + reduce grid: tests + bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stem_pool.py \
  > gpurun_out/r5/b26_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b26_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 200 python -u bench.py > gpurun_out/r5/b26_quad_$i.log 2>&1 || exit 10
  ZOO_POOL_QUAD=0 $T 200 python -u bench.py > gpurun_out/r5/b26_noquad_$i.log 2>&1 || exit 11
  ZOO_POOL_RED_BLOCKS=2048 $T 200 python -u bench.py > gpurun_out/r5/b26_red2048_$i.log 2>&1 || exit 12
done
for f in gpurun_out/r5/b26_{quad,noquad,red2048}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"final_loss": [0-9.]*' $f)"; done
cd /tmp && $T 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5/b26_prof" -o prof -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/r5/b26_prof.log" 2>&1 || exit 13
find "$GRAFT_REPO_ROOT/gpurun_out/r5/b26_prof" -name "*kernel_stats.csv" | head -1 | xargs grep -i "maxpool"
