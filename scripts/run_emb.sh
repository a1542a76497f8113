set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_emb.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 10 > gpurun_out/bert_train_emb.log 2>&1 || exit 2
$T 200 python bench.py --model ncf > gpurun_out/bench_ncf.log 2>&1 || exit 3
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ncf -o ncf -- python3 bench.py --model ncf --steps 20 --warmup 5 > gpurun_out/prof_ncf.log 2>&1 || exit 4
$T 200 python bench.py --batch 512 --steps 10 --warmup 4 > gpurun_out/bench_b512.log 2>&1 || exit 5
