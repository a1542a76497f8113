set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
for i in 1 2; do
ZOO_RESID_GRAD_FUSE=0 $T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 > gpurun_out/bert_res_off$i.log 2>&1 || exit 1
ZOO_RESID_GRAD_FUSE=1 $T 300 python analytics-zoo_amd/tools/bert_train.py --batch 128 --iters 20 > gpurun_out/bert_res_on$i.log 2>&1 || exit 2
done
