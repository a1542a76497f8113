set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_reentry.log 2>&1 || exit 1
$T 300 python bench.py > gpurun_out/bench_reentry.log 2>&1 || exit 2
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reentry -o rn -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/bench_prof_reentry.log 2>&1 || exit 3
