set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_bmm.py tests/test_gpu_zoo_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ssd.log 2>&1 || exit 1
