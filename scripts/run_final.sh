set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || exit 1
$T 200 python bench.py > gpurun_out/bench_final1.log 2>&1 || exit 2
$T 200 python bench.py > gpurun_out/bench_final2.log 2>&1 || exit 3
$T 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 4
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o rn -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/bench_prof_final.log 2>&1 || exit 5
