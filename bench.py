#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 (224x224, bf16) synchronous data-parallel
training throughput in images/sec for the whole node; ``--model ncf`` gives
the NCF records/sec metric (BASELINE.json).

  python bench.py --gpus N --steps K --warmup W [--batch 256] [--model resnet50|ncf]

For N > 1 one rank runs per GPU. Either launch the ranks yourself:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
or run ``python bench.py --gpus N`` directly: without WORLD_SIZE in the environment the
process does not touch the GPU, starts ``torch.distributed.run`` with N ranks as a child
process (never exec) and exits with its return code. A launched job whose world size is
not ``--gpus`` exits non-zero instead of reporting a mislabeled number.

Multi-GPU defaults are BigDL's: 16-bit (bf16) gradient wire with fp32 accumulation
(``ZOO_GRAD_COMPRESSION=auto``), 32 MB buckets for ResNet-50, one bucket for NCF.

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
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "analytics-zoo_amd"))

BASELINE_METRIC = "images/sec (whole node) ResNet-50 bf16"
BASELINE_VALUE = None  # BASELINE.json "published" is empty -> vs_baseline null


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "ncf", "mlp"],
                    help="mlp: a small CPU-capable dry-run model for launcher/DP tests (not a benchmark)")
    ap.add_argument("--sharded", action="store_true", help="ZeRO-1 sharded optimizer (BigDL AllReduceParameter)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the bucketed RCCL path even at world size 1 (implied by --sharded)")
    ap.add_argument("--grad-compression", default="auto", choices=["auto", "", "none", "bf16"],
                    help="gradient wire: auto = bf16 whenever GPU collectives run (BigDL 16-bit transfer)")
    ap.add_argument("--bucket-mb", type=float, default=0.0, help="0: per-model default (ResNet 32, NCF one bucket)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--comm", default="auto", choices=["auto", "torch", "native"],
                    help="bucket collectives through the torch ProcessGroup or the C++ RCCL layer; auto: native for "
                         "NCF (its captured step then holds the collectives and the update: one replay per step)")
    ap.add_argument("--input", default="auto", choices=["auto", "device", "featureset"],
                    help="featureset: ResNet-50 trained through NNEstimator.fit on a synthetic DataFrame of uint8 "
                         "NHWC images (FeatureSet -> pinned batches -> copy stream -> on-device normalisation), "
                         "BASELINE config 2; device: one device-resident fp32 batch reused every step; "
                         "auto (default): featureset for ResNet-50, device for the other models")
    a = ap.parse_args()
    if a.input == "auto":
        a.input = "featureset" if a.model == "resnet50" else "device"
    return a


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def build_resnet50(ctx, batch):
    import torch
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
    eng = TrainingEngine(model, softmax_cross_entropy, optim, bucket_mb=a_bucket(32.0))
    dev = ctx.device
    g = torch.Generator(device=dev)
    g.manual_seed(ctx.rank)
    x = torch.randn(batch, 3, 224, 224, device=dev, generator=g)
    y = torch.randint(0, 1000, (batch,), device=dev, generator=g)
    return eng, (x, y), "ResNet-50", {"image_size": 224, "optimizer": "SGD(nesterov, momentum=0.9, wd=1e-4, warmup 0.01->0.1/10 it)"}


def build_ncf(ctx, batch):
    import torch
    from zoo.models.recommendation.neuralcf import NeuralCF
    from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine

    torch.manual_seed(1234)
    users, items = 138493, 26744  # ml-20m shape
    model = NeuralCF(users, items, 5, user_embed=20, item_embed=20, hidden_layers=(40, 20, 10), include_mf=True,
                     mf_embed=20)
    # NCF's step is ~130 small kernels: capture forward+backward as one hipGraph
    # the whole gradient (26 MB fp32) in ONE bucket: NCF's backward is ~0.1 ms, too short to overlap
    eng = TrainingEngine(model, SparseCategoricalCrossEntropy(), Adam(lr=1e-3), hip_graph=True,
                         bucket_mb=a_bucket(1024.0))
    dev = ctx.device
    g = torch.Generator(device=dev)
    g.manual_seed(ctx.rank)
    u = torch.randint(1, users + 1, (batch,), device=dev, generator=g)
    i = torch.randint(1, items + 1, (batch,), device=dev, generator=g)
    x = torch.stack([u, i], 1)
    y = torch.randint(0, 5, (batch,), device=dev, generator=g)
    return eng, (x, y), "NCF", {"users": users, "items": items, "embed": 20, "hidden": [40, 20, 10]}


def build_mlp(ctx, batch):
    """Dry-run model (CPU/gloo capable): exercises launcher, ranks, DP sync and the JSON line."""
    import torch
    import torch.nn as nn
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    torch.manual_seed(1234)
    model = nn.Sequential(nn.Linear(64, 256), nn.Tanh(), nn.Linear(256, 256), nn.Tanh(), nn.Linear(256, 1))
    eng = TrainingEngine(model, MeanSquaredError(), SGD(learningrate=0.01, momentum=0.9),
                         bucket_mb=a_bucket(0.25))
    g = torch.Generator(device=ctx.device)
    g.manual_seed(ctx.rank)
    x = torch.randn(batch, 64, device=ctx.device, generator=g)
    y = torch.randn(batch, 1, device=ctx.device, generator=g)
    return eng, (x, y), "MLP-dry-run", {"note": "launcher/DP dry-run model, not a benchmark"}


_BUCKET = [0.0]


def a_bucket(default):
    return _BUCKET[0] if _BUCKET[0] > 0 else default


def run_featureset(a, ctx, world):
    """ResNet-50 through NNEstimator.fit (NNEstimator.scala:382-470): a pandas DataFrame of uint8
    224x224x3 images -> FeatureSet (native gather into pinned batches) -> the engine's copy
    stream (one batch ahead) -> uint8 normalisation fused into the stem. Times EXACTLY the K
    iterations after W warm-up iterations (device sync + barrier at both ends, from a per-
    iteration callback); returns (elapsed seconds, first loss, final loss, engine)."""
    import numpy as np
    import pandas as pd
    import torch
    import torch.distributed as dist
    from zoo.common.triggers import MaxIteration
    from zoo.feature.common import Lambda
    from zoo.models.image.resnet import resnet50
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD, EpochDecayWithWarmUp
    from zoo.pipeline.nnframes.nn_classifier import NNEstimator
    torch.manual_seed(1234)
    model = resnet50(num_classes=1000, zero_init_residual=True)
    warm = 10
    optim = SGD(learningrate=0.01, momentum=0.9, weightdecay=1e-4, dampening=0.0, nesterov=True,
                learningrate_schedule=EpochDecayWithWarmUp(warm, (0.1 - 0.01) / warm, lambda epoch: 0))
    # each rank builds only ITS partition of the DataFrame (a Spark partition on its executor):
    # one epoch covers the whole run, so no epoch edge falls inside the timed steps
    n = a.batch * (a.warmup + a.steps)
    rng = np.random.default_rng(4321 + 7 * ctx.rank)
    # a pool of two batches of distinct labelled images, repeated over the run's rows: every row is
    # still gathered into a pinned batch and copied to the GPU, and the model sees each image ~12
    # times, so the loss falls as on the device-resident bench (fully random rows give a random
    # label stream with nothing to fit: the loss rose)
    pool = min(n, 2 * a.batch)
    imgs = rng.integers(0, 256, size=(pool, 224, 224, 3), dtype=np.uint8)
    plabels = rng.integers(0, 1000, size=pool)
    pick = np.arange(n) % pool
    df = pd.DataFrame({"features": [imgs[i] for i in pick], "label": plabels[pick]})
    est = NNEstimator(model, softmax_cross_entropy, Lambda(lambda v: v), Lambda(lambda v: np.int64(v)))
    est.setBatchSize(a.batch * world).setOptimMethod(optim).setEndWhen(MaxIteration(a.warmup + a.steps))
    est.setLocalPartition(True)
    dev = ctx.device
    mark = {}

    def timer(eng, state):
        it = state["neval"] - 1
        # this iteration's device loss (a log_every flush has already moved it to the host)
        cur = eng._pending_loss[-1][1] if eng._pending_loss else torch.tensor(state["Loss"])
        if it == 1:
            mark["first"] = cur
        if it in (a.warmup, a.warmup + a.steps):
            _sync(dev)
            if world > 1:
                dist.barrier()
            _sync(dev)
            mark[it] = time.perf_counter()
            mark["last"] = cur
    est._train_callbacks = (timer,)
    est.fit(df)
    elapsed = mark[a.warmup + a.steps] - mark[a.warmup]
    return elapsed, mark.get("first"), mark.get("last"), est.engine


def grad_sync_label(eng, a):
    """What the gradient synchronisation actually did: "none" when no collective runs."""
    if not eng.sync.comm:
        return "none"
    lab = "sharded(ZeRO-1,bf16-weight-gather)" if eng.sync.mode == "sharded" else "allreduce(bucketed,overlapped)"
    return lab + ("+bf16-wire" if eng.sync.compress else "+fp32-wire") + \
        ",%d-buckets" % len(eng.sync.buckets) + (",native-comm" if eng.sync.ncomm is not None else "") + \
        (",whole-step-hipgraph" if getattr(eng, "full_graph", False) else "")


def comm_diagnostics(eng, x, y, world):
    """Self-check fields for multi-GPU runs (measured AFTER the timed steps, so the event
    timing does not perturb them): RCCL world size, cross-rank max |difference| of a checksum
    of the fp32 master weights (0 = every rank holds the same model), exposed comm time per
    step (the compute stream's wait on the comm stream) and per-bucket bus bandwidth."""
    import torch
    import torch.distributed as dist
    sync = eng.sync
    if not sync.comm:
        return {"rccl_world": 1}
    sync.collect_stats = True
    for _ in range(3):
        eng.train_step(x, y)
    _sync(x.device)
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(a):
    """--gpus N > 1 without a launcher: start N ranks with torch.distributed.run as a CHILD
    process. This process has not touched the GPU (no torch.cuda call, no HIP context) and
    never execs; it waits and returns the child's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL between the ranks
    print("bench.py: launching %d ranks: %s" % (a.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(a)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != a.gpus:
        print("bench.py: --gpus %d but the job has WORLD_SIZE=%d ranks; refusing to report a "
              "mislabeled number" % (a.gpus, world_env), file=sys.stderr, flush=True)
        return 2
    _BUCKET[0] = a.bucket_mb
    import torch
    import torch.distributed as dist
    from zoo.common.nncontext import init_nncontext
    comp = "" if a.grad_compression == "none" else a.grad_compression
    comm = a.comm if a.comm != "auto" else ("native" if a.model == "ncf" else "torch")
    ctx = init_nncontext("bench", sharded_optimizer=a.sharded, force_comm=a.force_comm or a.sharded,
                         grad_compression=comp, comm=comm)
    world = ctx.world_size
    if world != a.gpus:
        print("bench.py: --gpus %d but the process group has %d ranks" % (a.gpus, world), file=sys.stderr)
        return 2
    dev = ctx.device
    if a.input == "featureset":
        if a.model != "resnet50":
            print("bench.py: --input featureset is the ResNet-50 NNEstimator config", file=sys.stderr)
            return 2
        elapsed, first_loss, loss, eng = run_featureset(a, ctx, world)
        return report(a, ctx, world, dev, eng, None, None, elapsed, first_loss, loss, 0.0, a.batch,
                      BASELINE_METRIC, "images/sec", "ResNet-50",
                      {"image_size": 224, "optimizer": "SGD(nesterov, momentum=0.9, wd=1e-4, warmup 0.01->0.1/10 it)",
                       "input": "featureset"},
                      "synthetic uint8 NHWC images in a pandas DataFrame (a pool of 2 x batch distinct "
                      "labelled images per rank repeated over the rows) -> NNEstimator.fit (FeatureSet, "
                      "pinned batches, copy stream); random-init weights")
    if a.model == "resnet50":
        batch = a.batch
        eng, (x, y), model_name, extra = build_resnet50(ctx, batch)
        metric, unit = BASELINE_METRIC, "images/sec"
    elif a.model == "ncf":
        batch = a.batch if a.batch != 256 else 65536
        eng, (x, y), model_name, extra = build_ncf(ctx, batch)
        metric, unit = "records/sec (whole node) NCF", "records/sec"
    else:
        batch = a.batch
        eng, (x, y), model_name, extra = build_mlp(ctx, batch)
        metric, unit = "samples/sec (dry-run MLP, not a benchmark)", "samples/sec"

    first_loss = None
    for _ in range(a.warmup):
        l0 = eng.train_step(x, y)
        if first_loss is None:
            first_loss = l0
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(a.steps):
        h0 = time.perf_counter()
        loss = eng.train_step(x, y)
        host += time.perf_counter() - h0
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    elapsed = time.perf_counter() - t0
    return report(a, ctx, world, dev, eng, x, y, elapsed, first_loss, loss, host, batch, metric, unit, model_name,
                  extra, "synthetic (random-init weights, random inputs/labels)")


def report(a, ctx, world, dev, eng, x, y, elapsed, first_loss, loss, host, batch, metric, unit, model_name, extra,
           data):
    """Max elapsed over ranks -> rank 0 prints the one JSON line."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = float(loss.float().item()) if loss is not None else None
    diag = comm_diagnostics(eng, x, y, world) if x is not None else {"rccl_world": world}
    total = batch * world * a.steps
    value = total / elapsed
    if ctx.rank == 0:
        out = {
            "metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": data,
            "config": dict({"model": model_name, "global_batch": batch * world, "per_gpu_batch": batch,
                            "seq_len": None, "parallelism": "dp%d" % world,
                            "grad_sync": grad_sync_label(eng, a)},
                           **extra),
            "first_loss": round(float(first_loss.float().item()), 4) if first_loss is not None else None,
            "final_loss": round(final_loss, 4) if final_loss is not None else None,
        }
        if x is not None:
            # issue time of a step on the host (no device sync inside the timed loop): near
            # ms_per_step means host-bound, well below means device-bound
            out["host_ms_per_step"] = round(host / a.steps * 1e3, 3)
        out.update(diag)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
