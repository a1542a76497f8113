#!/bin/bash
# MFMA probe, BERT parity test, serving suite (1 GPU)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/misc
timeout -k 5 60 ./analytics-zoo_amd/tools/mfma_probe > gpurun_out/misc/probe.log 2>&1; cat gpurun_out/misc/probe.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_bert_parity.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/misc/bert_parity.log 2>&1
echo "bert parity rc=$?"; tail -6 gpurun_out/misc/bert_parity.log
timeout -k 10 500 python -u analytics-zoo_amd/tools/serving_bench.py suite --duration 6 --out gpurun_out/misc/suite.json > gpurun_out/misc/suite.log 2>&1
echo "suite rc=$?"; grep bench gpurun_out/misc/suite.log | tail -14
timeout -k 10 200 python -u analytics-zoo_amd/tools/glue_report.py --model ncf --steps 3 > gpurun_out/misc/ncf_glue.log 2>&1
echo "ncf glue rc=$?"; head -40 gpurun_out/misc/ncf_glue.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_convlstm_seq.py tests/test_gpu_keras_native.py -x -q -k "convlstm or ConvLSTM" --timeout 120 --timeout-method thread > gpurun_out/misc/convlstm_test.log 2>&1
echo "convlstm tests rc=$?"; tail -4 gpurun_out/misc/convlstm_test.log
timeout -k 10 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/misc/convlstm_bench.log 2>&1
echo "convlstm bench rc=$?"; tail -2 gpurun_out/misc/convlstm_bench.log
