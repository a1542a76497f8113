#!/usr/bin/env python3
"""ResNet ImageNet training (Zs/examples/resnet/TrainImageNet.scala + Utils.scala).

The reference recipe: SGD momentum 0.9 (nesterov), weight decay 1e-4, batch 8192 over the
cluster, EpochDecayWithWarmUp (linear warm-up to lr*batch/256, then step decay /10 at
epochs 30/60/80), zero-initialised last BN gamma per block, optional SyncBN. Here the data
is a synthetic ImageNet (random images and labels -- no dataset download), the model the
native NHWC ResNet (hand-written HIP conv/BN kernels on MI355X), and distribution one
process per GPU over RCCL:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        examples/resnet/train_imagenet.py --batch 256 --iters 100 --sync-bn

Checkpoints (``--checkpoint DIR``) are written in the BigDL ``.model`` format with the
optimizer state, every ``--checkpoint-every`` iterations.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--depth", type=int, default=50, choices=[18, 34, 50, 101, 152])
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--batch", type=int, default=256, help="per-process batch")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--lr", type=float, default=0.1, help="peak learning rate for batch 256")
    ap.add_argument("--warmup-iters", type=int, default=10)
    ap.add_argument("--sync-bn", action="store_true")
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--width", type=int, default=64, help="stem width (64 = the standard ResNet)")
    a = ap.parse_args(argv)

    import torch
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import ResNet, BasicBlock, Bottleneck
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD, EpochDecayWithWarmUp
    from zoo.pipeline.engine import TrainingEngine

    ctx = init_nncontext("train_imagenet")
    if a.sync_bn:
        from zoo.parallel.sync_bn import set_sync_bn
        set_sync_bn(True)
    layers = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}[a.depth]
    block = BasicBlock if a.depth < 50 else Bottleneck
    torch.manual_seed(1234)
    model = ResNet(block, layers, num_classes=a.classes, width=a.width, zero_init_residual=True)
    peak = a.lr * a.batch * ctx.world_size / 256.0
    warm = max(1, a.warmup_iters)
    sched = EpochDecayWithWarmUp(warm, (peak - a.lr / 10) / warm, lambda epoch: 0)
    optim = SGD(learningrate=a.lr / 10, momentum=0.9, weightdecay=1e-4, dampening=0.0, nesterov=True,
                learningrate_schedule=sched)
    eng = TrainingEngine(model, softmax_cross_entropy, optim)
    if a.checkpoint:
        eng.set_checkpoint(a.checkpoint, overwrite=False)
    g = torch.Generator(device=ctx.device)
    g.manual_seed(ctx.rank)
    x = torch.randn(a.batch, 3, a.image_size, a.image_size, device=ctx.device, generator=g)
    y = torch.randint(0, a.classes, (a.batch,), device=ctx.device, generator=g)
    t0, losses = time.perf_counter(), []
    for it in range(1, a.iters + 1):
        loss = eng.train_step(x, y)
        if it % 10 == 0 or it == a.iters:
            losses.append(float(loss))
            if ctx.rank == 0:
                dt = time.perf_counter() - t0
                print("iter %d loss %.4f  %.1f img/s" % (it, losses[-1], it * a.batch * ctx.world_size / dt),
                      flush=True)
        if a.checkpoint and a.checkpoint_every and it % a.checkpoint_every == 0:
            eng.save_checkpoint()
    return losses


if __name__ == "__main__":
    main()
