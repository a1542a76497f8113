#!/bin/bash
# r6 A/B 2: full GPU suite after the knob pruning; ResNet-50 default (featureset) vs device pair
# with the new defaults; BERT-base b128: side stream on/off x native / hipBLASLt linears
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/ab2_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab2_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  $T 300 python -u bench.py > gpurun_out/r6/ab2_fs_$i.log 2>&1 || exit 21
  tail -1 gpurun_out/r6/ab2_fs_$i.log | cut -c1-200
  $T 300 python -u bench.py --input device > gpurun_out/r6/ab2_dev_$i.log 2>&1 || exit 22
  tail -1 gpurun_out/r6/ab2_dev_$i.log | cut -c1-200
done
bert() {  # tag, env...
  local tag=$1; shift
  env "$@" $T 300 python3 -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 > gpurun_out/r6/ab2_bert_$tag.log 2>&1 || exit 30
  echo "$tag $(tail -1 gpurun_out/r6/ab2_bert_$tag.log)"
}
for i in 1 2; do
  bert base$i
  bert noside$i ZOO_WGRAD_STREAM=0
  bert blas$i ZOO_LINEAR_BLAS=1
  bert blasnoside$i ZOO_LINEAR_BLAS=1 ZOO_WGRAD_STREAM=0
done
