set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
run() { echo "== $1" >> gpurun_out/knobs.log; env $1 $T 200 python bench.py --steps 20 --warmup 5 2>&1 | tail -1 >> gpurun_out/knobs.log; }
rm -f gpurun_out/knobs.log
run "ZOO_X=0" || exit 1
run "ZOO_WGRAD_WG=512" || exit 1
run "ZOO_WGRAD_WG=768" || exit 1
run "ZOO_WGRAD_WG=2048" || exit 1
run "ZOO_WGRAD_MINPIX=1024" || exit 1
run "ZOO_WGRAD_PARTIAL_MB=64" || exit 1
run "ZOO_WGRAD_PARTIAL_MB=4" || exit 1
