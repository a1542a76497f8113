#!/bin/bash
# r5 batch 59: model-zoo throughput refresh (ImageClassifier backbones + SSD-300, NCF bench)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u analytics-zoo_amd/tools/zoo_models_bench.py --batch 64 --steps 10 > gpurun_out/r5/b59_zoo_models.log 2>&1 || exit 10
grep "{" gpurun_out/r5/b59_zoo_models.log | cut -c1-200
