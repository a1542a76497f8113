#!/bin/bash
# r5 batch 67: dropout seed staged only for graphs that read it: graph / dropout tests + NCF + BERT graph
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ibo.py tests/test_gpu_graph_shapes.py \
  tests/test_gpu_kernels.py -k "graph or dropout or ibo or shapes" > gpurun_out/r5/b67_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b67_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 300 python -u bench.py --model ncf --batch 65536 --steps 100 --warmup 20 > gpurun_out/r5/b67_ncf_$i.log 2>&1 || exit 10
done
for f in gpurun_out/r5/b67_ncf_?.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
