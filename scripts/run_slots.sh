set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_nets.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_slots.log 2>&1 || exit 1
rm -f gpurun_out/slots.log
for v in 0 512 2048 8192; do echo "== $v" >> gpurun_out/slots.log; ZOO_STAT_SLOT_MIN_TILES=$v $T 200 python bench.py --steps 20 --warmup 5 2>&1 | tail -1 >> gpurun_out/slots.log || exit 2; done
