set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_tfnet.py tests/test_openvino.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_misc.log 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn_final -o rn -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_rn_final.log 2>&1 || exit 2
