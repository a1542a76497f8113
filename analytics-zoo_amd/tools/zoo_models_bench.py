#!/usr/bin/env python3
"""Model-zoo throughput on the native NHWC kernels: ImageClassifier backbones
(inference and training) and SSD-300 training, synthetic data, bf16.

  python tools/zoo_models_bench.py [--models mobilenet,ssd300] [--batch 64] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def sync():
    torch.cuda.synchronize()


def bench_infer(name, batch, steps, hw):
    from zoo.models.image.imageclassification.nets import build
    m = build(name, 1000).cuda().eval()
    x = torch.randn(batch, 3, hw, hw, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            m(x)
        sync()
        t = time.perf_counter()
        for _ in range(steps):
            m(x)
        sync()
    dt = (time.perf_counter() - t) / steps
    return {"model": name, "mode": "inference", "batch": batch, "ms": dt * 1e3, "img_s": batch / dt}


def bench_train(name, batch, steps, hw):
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.imageclassification.nets import build
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("zoo-bench")
    eng = TrainingEngine(build(name, 1000), softmax_cross_entropy, SGD(learningrate=0.01, momentum=0.9))
    x = torch.randn(batch, 3, hw, hw, device="cuda")
    y = torch.randint(0, 1000, (batch,), device="cuda")
    for _ in range(3):
        eng.train_step(x, y)
    sync()
    t = time.perf_counter()
    for _ in range(steps):
        loss = eng.train_step(x, y)
    sync()
    dt = (time.perf_counter() - t) / steps
    return {"model": name, "mode": "train", "batch": batch, "ms": dt * 1e3, "img_s": batch / dt,
            "loss": float(loss.item())}


def bench_ssd(batch, steps, mobilenet=False):
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.objectdetection.ssd import SSD, SSDMobileNet, MultiBoxLoss
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("zoo-bench")
    model = SSDMobileNet(21) if mobilenet else SSD(21)
    crit = MultiBoxLoss(21)
    pri = model.priors

    def loss_fn(out, targets):
        return crit(out[0], out[1], pri.to(out[0].device), targets)
    eng = TrainingEngine(model, loss_fn, SGD(learningrate=1e-3, momentum=0.9))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(batch, 3, 300, 300, device="cuda")
    targets = []
    for _ in range(batch):
        n = 3
        xy = torch.rand(n, 2, generator=g) * 0.6
        wh = torch.rand(n, 2, generator=g) * 0.3 + 0.05
        lab = torch.randint(1, 21, (n, 1), generator=g).float()
        targets.append(torch.cat([lab, xy, xy + wh], 1).cuda())
    for _ in range(2):
        eng.train_step(x, targets)
    sync()
    t = time.perf_counter()
    for _ in range(steps):
        loss = eng.train_step(x, targets)
    sync()
    dt = (time.perf_counter() - t) / steps
    return {"model": "ssd-mobilenet-300" if mobilenet else "ssd-vgg16-300", "mode": "train", "batch": batch,
            "ms": dt * 1e3, "img_s": batch / dt, "loss": float(loss.item())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="mobilenet,mobilenet-v2,inception-v1,vgg-16,ssd300")
    ap.add_argument("--mode", default="infer,train")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    for name in a.models.split(","):
        if name.startswith("ssd"):
            print(json.dumps(bench_ssd(min(a.batch, 32), a.steps, mobilenet="mobile" in name)), flush=True)
            continue
        hw = 299 if name == "inception-v3" else (227 if name in ("alexnet", "squeezenet") else 224)
        if "infer" in a.mode:
            print(json.dumps(bench_infer(name, a.batch, a.steps, hw)), flush=True)
        if "train" in a.mode:
            print(json.dumps(bench_train(name, a.batch, a.steps, hw)), flush=True)


if __name__ == "__main__":
    main()
