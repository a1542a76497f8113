#!/bin/bash
# r5 batch 66: in-backward optimizer opt-in under capture: IBO / graph tests + NCF bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ibo.py tests/test_gpu_graph_shapes.py \
  > gpurun_out/r5/b66_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b66_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 300 python -u bench.py --model ncf --batch 65536 --steps 100 --warmup 20 > gpurun_out/r5/b66_ncf_$i.log 2>&1 || exit 10
done
for f in gpurun_out/r5/b66_ncf_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
