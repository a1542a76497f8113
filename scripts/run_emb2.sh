set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_embedding.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_emb.log 2>&1 || exit 1
$T 120 python analytics-zoo_amd/tools/emb_bench.py > gpurun_out/emb_bench.log 2>&1 || exit 2
$T 200 python bench.py --model ncf > gpurun_out/bench_ncf.log 2>&1 || exit 3
$T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_train_emb.log 2>&1 || exit 4
