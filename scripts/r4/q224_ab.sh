#!/bin/bash
# igemm2 224x256 wave-quantization tile: numerics, conv / linear A/B, end to end
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/q224; mkdir -p $O
ZOO_I2_TEST_224=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_igemm2.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 2
for q in 1 0; do
  ZOO_I2_Q224=$q timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops fwd,dgrad > $O/sweep_q$q.log 2>&1 || exit 3
  echo "q224=$q $(tail -1 $O/sweep_q$q.log)"
  ZOO_I2_Q224=$q timeout -k 10 200 python -u analytics-zoo_amd/tools/linear_epi_bench.py > $O/lin_q$q.log 2>&1 || exit 4
  grep "^{" $O/lin_q$q.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('  lin', r['gemm'], 'lean', r['us_lean'], 'bias', r['us_bias'])"
done
for i in 1 2; do
  for q in 1 0; do
    ZOO_I2_Q224=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/rn_q${q}_$i.log 2>&1 || exit 5
    echo "resnet q224=$q run=$i $(grep -o '"value": [0-9.]*' $O/rn_q${q}_$i.log)"
    ZOO_I2_Q224=$q timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/bert_q${q}_$i.log 2>&1 || exit 6
    echo "bert q224=$q run=$i $(tail -1 $O/bert_q${q}_$i.log | cut -c1-100)"
  done
done
