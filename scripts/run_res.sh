set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_residual_grad.py tests/test_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_res.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_train_res.log 2>&1 || exit 2
