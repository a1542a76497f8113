#!/bin/bash
# igemm2 software-pipelined 2-stage loop: numerics, GEMM / conv A/B (ZOO_I2_PIPE 0 / 1), end to end
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pipe; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_igemm2.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 2
for p in 1 0; do
  ZOO_I2_PIPE=$p timeout -k 10 200 python -u analytics-zoo_amd/tools/linear_epi_bench.py > $O/lin_p$p.log 2>&1 || exit 6
  echo "pipe=$p linear:"; grep "^{" $O/lin_p$p.log | cut -c1-220
done
for p in 1 0; do
  ZOO_I2_PIPE=$p timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops fwd,dgrad > $O/sweep_p$p.log 2>&1 || exit 3
  echo "pipe=$p $(tail -1 $O/sweep_p$p.log)"
done
for p in 1 0; do
  ZOO_I2_PIPE=$p timeout -k 10 240 python -u analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 30 > $O/bert_p$p.log 2>&1 || exit 4
  echo "bert pipe=$p $(tail -1 $O/bert_p$p.log)"
done
for p in 1 0; do
  ZOO_I2_PIPE=$p timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/rn_p$p.log 2>&1 || exit 5
  echo "resnet pipe=$p $(grep -o '"value": [0-9.]*' $O/rn_p$p.log) $(grep -o '"final_loss": [0-9.]*' $O/rn_p$p.log)"
done
