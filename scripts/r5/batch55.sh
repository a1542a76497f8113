#!/bin/bash
# r5 batch 55: the driver's torchrun launch path at N = 1 (rendezvous, RCCL world 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r5/b55_torchrun.log 2>&1 || exit 10
grep '"metric"' gpurun_out/r5/b55_torchrun.log
