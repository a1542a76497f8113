set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model ncf > gpurun_out/bench_ncf_final.log 2>&1 || exit 1
