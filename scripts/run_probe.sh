set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 120 python analytics-zoo_amd/tools/conv1x1_probe.py > gpurun_out/probe_default.log 2>&1 || exit 1
ZOO_IGEMM_BN=128 $T 120 python analytics-zoo_amd/tools/conv1x1_probe.py > gpurun_out/probe_bn128.log 2>&1 || exit 2
ZOO_IGEMM_DMA=0 $T 120 python analytics-zoo_amd/tools/conv1x1_probe.py > gpurun_out/probe_nodma.log 2>&1 || exit 3
$T 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_probe -o probe -- python analytics-zoo_amd/tools/conv1x1_probe.py --shapes "56,64,256;56,256,64" --iters 10 > gpurun_out/probe_prof.log 2>&1 || exit 4
