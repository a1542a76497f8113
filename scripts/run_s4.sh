set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python bench.py --steps 20 --warmup 15 > gpurun_out/bench_s4e.log 2>&1 || exit 2
ZOO_FLIP_CACHE=0 $T 300 python bench.py --steps 20 --warmup 15 > gpurun_out/bench_s4e_noflipcache.log 2>&1 || exit 3
$T 300 python bench.py --steps 20 --warmup 15 > gpurun_out/bench_s4e2.log 2>&1 || exit 4
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s4e -o bench -- python3 bench.py --steps 15 --warmup 5 > gpurun_out/prof_s4e.log 2>&1 || exit 5
