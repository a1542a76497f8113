set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_stem_pool.py tests/test_gpu_zoo_kernels.py tests/test_gpu_kernels.py tests/test_gpu_resnet50_parity.py -x -q --timeout 120 -s --timeout-method thread > gpurun_out/pytest_stem.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
for i in 1 2; do
ZOO_FUSE_STEM_POOL=0 $T 200 python bench.py > gpurun_out/bench_stem_off$i.log 2>&1 || exit 2
ZOO_FUSE_STEM_POOL=1 $T 200 python bench.py > gpurun_out/bench_stem_on$i.log 2>&1 || exit 3
done
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stem -o rn -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/bench_prof_stem.log 2>&1 || exit 4
