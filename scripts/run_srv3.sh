set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python analytics-zoo_amd/tools/serving_bench.py e2e --model bert --batch 128 --images 16384 --client-procs 6 > gpurun_out/serving_bert_e2e_procs.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/serving_bench.py e2e --batch 128 --images 8192 --client-procs 6 > gpurun_out/serving_rn_e2e_procs.log 2>&1 || exit 2
