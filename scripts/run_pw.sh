set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_pointwise.py tests/test_gpu_wgrad256.py tests/test_openvino.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pw.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_train_pw.log 2>&1 || exit 2
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert4 -o bert -- python3 analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/prof_bert4.log 2>&1 || exit 3
