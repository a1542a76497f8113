set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sparse.log 2>&1 || exit 1
$T 200 python analytics-zoo_amd/tools/wnd_bench.py --batch 8192 --steps 30 > gpurun_out/wnd_bench.log 2>&1 || exit 2
$T 200 python analytics-zoo_amd/tools/wnd_bench.py --batch 65536 --steps 20 >> gpurun_out/wnd_bench.log 2>&1 || exit 3
$T 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wnd -o wnd -- python3 analytics-zoo_amd/tools/wnd_bench.py --batch 8192 --steps 20 > gpurun_out/prof_wnd.log 2>&1 || exit 4
