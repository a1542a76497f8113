#!/usr/bin/env python3
"""Inception-v1 training (pyzoo/zoo/examples/inception/inception.py): the GoogLeNet (BN)
backbone of the ImageClassifier zoo, trained with SGD + momentum and a poly learning-rate
schedule by the framework's TrainingEngine (flat fp32 master weights, fused native optimizer,
one hipGraph per step on the GPU; DDP over RCCL when launched with torchrun). Synthetic
ImageNet-shaped data here (--image-size 224 for the real geometry)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401


def main(argv=None):
    ap = _common.add_common(argparse.ArgumentParser(description=__doc__.split("\n")[0]))
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.0896)
    a = ap.parse_args(argv)
    import torch
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.imageclassification.nets import build
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD, Poly
    from zoo.pipeline.engine import TrainingEngine
    ctx = init_nncontext("inception-v1")
    torch.manual_seed(a.seed)
    dev = ctx.device
    eng = TrainingEngine(build("inception-v1", a.classes), softmax_cross_entropy,
                         SGD(learningrate=a.lr, momentum=0.9, weightdecay=1e-4,
                             leaningrate_schedule=Poly(0.5, max(a.iters, 1))))
    losses = []
    for it in range(a.iters):
        x = torch.randn(a.batch, 3, a.image_size, a.image_size, device=dev)
        y = torch.randint(0, a.classes, (a.batch,), device=dev)
        losses.append(float(eng.train_step(x, y).item()))
        print("iter %d loss %.4f" % (it, losses[-1]))
    return losses


if __name__ == "__main__":
    main()
