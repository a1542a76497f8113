#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 (224x224, bf16) synchronous data-parallel
training throughput in images/sec for the whole node; ``--model ncf`` gives
the NCF records/sec metric (BASELINE.json).

  python bench.py --gpus N --steps K --warmup W [--batch 256] [--model resnet50|ncf]

For N > 1 launch one rank per GPU:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Each step = synthetic batch -> NCHW->NHWC bf16 conversion -> forward ->
softmax cross-entropy -> backward -> RCCL gradient all-reduce (bucketed,
overlapped) -> fused SGD-momentum update of the fp32 master weights + bf16
copy. Weak scaling: the per-GPU batch is fixed, global batch = batch * N.
Timing: W untimed warmup steps, then barrier + device sync, K timed steps,
barrier + device sync; the max elapsed time over ranks is reported.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "analytics-zoo_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_METRIC = "images/sec (whole node) ResNet-50 bf16"
BASELINE_VALUE = None  # BASELINE.json "published" is empty -> vs_baseline null


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "ncf"])
    ap.add_argument("--sharded", action="store_true", help="ZeRO-1 sharded optimizer (BigDL AllReduceParameter)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the bucketed RCCL path even at world size 1 (implied by --sharded)")
    ap.add_argument("--grad-compression", default="", choices=["", "bf16"])
    ap.add_argument("--profile-steps", type=int, default=0)
    return ap.parse_args()


def build_resnet50(ctx, batch):
    from zoo.models.image.resnet import resnet50
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD, EpochDecayWithWarmUp
    from zoo.pipeline.engine import TrainingEngine

    torch.manual_seed(1234)
    # the reference ImageNet recipe (Zs/examples/resnet/TrainImageNet.scala:115-127 + Utils.scala:49-56):
    # SGD momentum 0.9 nesterov, wd 1e-4, EpochDecayWithWarmUp (here: 0.01 -> 0.1 over 10 iterations),
    # zero-initialised last BN gamma per block. Without warm-up the fixed-batch run diverges in plain
    # fp32 PyTorch too (profiles/resnet50_parity_r2.md), so the bench would time a diverging step.
    model = resnet50(num_classes=1000, zero_init_residual=True)
    warm = 10
    optim = SGD(learningrate=0.01, momentum=0.9, weightdecay=1e-4, dampening=0.0, nesterov=True,
                learningrate_schedule=EpochDecayWithWarmUp(warm, (0.1 - 0.01) / warm, lambda epoch: 0))
    eng = TrainingEngine(model, softmax_cross_entropy, optim)
    dev = ctx.device
    g = torch.Generator(device=dev)
    g.manual_seed(ctx.rank)
    x = torch.randn(batch, 3, 224, 224, device=dev, generator=g)
    y = torch.randint(0, 1000, (batch,), device=dev, generator=g)
    return eng, (x, y), "ResNet-50", {"image_size": 224, "optimizer": "SGD(nesterov, momentum=0.9, wd=1e-4, warmup 0.01->0.1/10 it)"}


def build_ncf(ctx, batch):
    from zoo.models.recommendation.neuralcf import NeuralCF
    from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine

    torch.manual_seed(1234)
    users, items = 138493, 26744  # ml-20m shape
    model = NeuralCF(users, items, 5, user_embed=20, item_embed=20, hidden_layers=(40, 20, 10), include_mf=True,
                     mf_embed=20)
    # NCF's step is ~130 small kernels: capture forward+backward as one hipGraph
    eng = TrainingEngine(model, SparseCategoricalCrossEntropy(), Adam(lr=1e-3), hip_graph=True)
    dev = ctx.device
    g = torch.Generator(device=dev)
    g.manual_seed(ctx.rank)
    u = torch.randint(1, users + 1, (batch,), device=dev, generator=g)
    i = torch.randint(1, items + 1, (batch,), device=dev, generator=g)
    x = torch.stack([u, i], 1)
    y = torch.randint(0, 5, (batch,), device=dev, generator=g)
    return eng, (x, y), "NCF", {"users": users, "items": items, "embed": 20, "hidden": [40, 20, 10]}


def grad_sync_label(eng, a):
    """What the gradient synchronisation actually did: "none" when no collective runs."""
    if not eng.sync.comm:
        return "none"
    lab = "sharded(ZeRO-1,bf16-weight-gather)" if eng.sync.mode == "sharded" else "allreduce(bucketed,overlapped)"
    return lab + ("+bf16-wire" if a.grad_compression else "")


def comm_diagnostics(eng, x, y, world):
    """Self-check fields for multi-GPU runs (measured AFTER the timed steps, so the event
    timing does not perturb them): RCCL world size, cross-rank max |difference| of a checksum
    of the fp32 master weights (0 = every rank holds the same model), exposed comm time per
    step (the compute stream's wait on the comm stream) and per-bucket bus bandwidth."""
    sync = eng.sync
    if not sync.comm:
        return {"rccl_world": 1}
    sync.collect_stats = True
    for _ in range(3):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    sync.collect_stats = False
    summ = sync.comm_summary()
    sync.sync_master()
    m = eng.flat.master.double()
    w = (torch.arange(m.numel(), device=m.device) % 1009 + 1).double()
    cs = torch.stack([m.sum(), (m * w).sum()])
    hi, lo = cs.clone(), cs.clone()
    if world > 1:
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    b = summ["buckets"]
    bus = [r["busbw_GBs"] for r in b if r["ms"] > 0]
    return {"rccl_world": dist.get_world_size() if dist.is_initialized() else 1,
            "comm_backend": dist.get_backend() if dist.is_initialized() else None,
            "master_checksum_maxdiff": float((hi - lo).abs().max().item()),
            "exposed_comm_ms_per_step": summ["exposed_comm_ms_per_step"],
            "comm_buckets": len(b), "comm_MB_per_step": round(sum(r["MB"] for r in b), 1),
            "bucket_busbw_GBs": {"mean": round(sum(bus) / len(bus), 1) if bus else 0.0,
                                 "max": max(bus) if bus else 0.0, "min": min(bus) if bus else 0.0}}


def main():
    a = parse()
    from zoo.common.nncontext import init_nncontext
    ctx = init_nncontext("bench", sharded_optimizer=a.sharded, force_comm=a.force_comm or a.sharded,
                         grad_compression=a.grad_compression)
    world = ctx.world_size
    if a.model == "resnet50":
        batch = a.batch
        eng, (x, y), model_name, extra = build_resnet50(ctx, batch)
        metric, unit = BASELINE_METRIC, "images/sec"
    else:
        batch = a.batch if a.batch != 256 else 65536
        eng, (x, y), model_name, extra = build_ncf(ctx, batch)
        metric, unit = "records/sec (whole node) NCF", "records/sec"

    first_loss = None
    for _ in range(a.warmup):
        l0 = eng.train_step(x, y)
        if first_loss is None:
            first_loss = l0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = eng.train_step(x, y)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=ctx.device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = float(loss.float().item())
    diag = comm_diagnostics(eng, x, y, world)
    total = batch * world * a.steps
    value = total / elapsed
    if ctx.rank == 0:
        out = {
            "metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "bf16", "data": "synthetic (random-init weights, random inputs/labels)",
            "config": dict({"model": model_name, "global_batch": batch * world, "per_gpu_batch": batch,
                            "seq_len": None, "parallelism": "dp%d" % world,
                            "grad_sync": grad_sync_label(eng, a)},
                           **extra),
            "first_loss": round(float(first_loss.float().item()), 4) if first_loss is not None else None,
            "final_loss": round(final_loss, 4),
        }
        out.update(diag)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
