set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_s4f.log 2>&1 || exit 1
$T 300 python bench.py --steps 20 --warmup 15 > gpurun_out/bench_s4f.log 2>&1 || exit 2
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s4f -o bench -- python3 bench.py --steps 15 --warmup 5 > gpurun_out/prof_s4f.log 2>&1 || exit 3
