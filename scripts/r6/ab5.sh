#!/bin/bash
# r6 run 5: 12-wave 256x192 igemm2 tile (numerics, isolated BERT GEMMs, BERT step forced) and the
# transposed band weight gradient of the stage-1 1x1 64->256 convs (numerics, ResNet-50 A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_igemm2.py tests/test_gpu_kernels.py tests/test_gpu_resnet50_parity.py \
  -k "igemm2 or band or resnet50" -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/ab5_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab5_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
$T 300 python3 -u analytics-zoo_amd/tools/gemm_bench.py --bert --tiles 0,5,11,12 > gpurun_out/r6/ab5_gemm_tiles.log 2>&1 || exit 23
grep '"M"' gpurun_out/r6/ab5_gemm_tiles.log | cut -c1-300
for i in 1 2; do
  for t in 0 12; do
    $T 300 python3 -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 --i2-tile $t > gpurun_out/r6/ab5_bert_t${t}_$i.log 2>&1 || exit 31
    echo "t$t $(tail -1 gpurun_out/r6/ab5_bert_t${t}_$i.log | cut -c1-120)"
  done
done
run() {  # tag, env...
  local tag=$1; shift
  env "$@" $T 300 python -u bench.py --input device > gpurun_out/r6/ab5_$tag.log 2>&1 || exit 21
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6/ab5_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
}
for i in 1 2 3; do
  run band2_$i ZOO_WGRAD_BAND=2
  run band1_$i ZOO_WGRAD_BAND=1
done
