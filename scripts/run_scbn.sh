set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_shortcut_bn.py tests/test_gpu_resnet50_parity.py tests/test_gpu_kernels.py tests/test_gpu_ddp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_scbn.log 2>&1 || exit 1
for i in 1 2; do
ZOO_FUSE_SHORTCUT_BN=0 $T 200 python bench.py > gpurun_out/bench_scbn_off$i.log 2>&1 || exit 2
ZOO_FUSE_SHORTCUT_BN=1 $T 200 python bench.py > gpurun_out/bench_scbn_on$i.log 2>&1 || exit 3
done
