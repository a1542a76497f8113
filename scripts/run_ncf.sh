set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 200 python bench.py --model ncf > gpurun_out/bench_ncf.log 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ncf -o ncf -- python3 bench.py --model ncf --steps 20 --warmup 5 > gpurun_out/prof_ncf.log 2>&1 || exit 2
$T 200 python bench.py --batch 512 --steps 10 --warmup 4 > gpurun_out/bench_b512.log 2>&1 || exit 3
