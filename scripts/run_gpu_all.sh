set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || exit 1
$T 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 2
$T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_train_final.log 2>&1 || exit 3
