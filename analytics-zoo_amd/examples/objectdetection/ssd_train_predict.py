#!/usr/bin/env python3
"""SSD object detection (pyzoo/zoo/examples/objectdetection/predict.py + the SSD training
of Zs/models/image/objectdetection): a few MultiBoxLoss training steps of SSD-300 on
synthetic images with random boxes, then detection output (decode + native NMS) and the
mean average precision of the detections. ``--backbone mobilenet`` for SSD-MobileNet."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--classes", type=int, default=4)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args(argv)
    import torch
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.objectdetection import SSD, DetectionOutputSSD, MultiBoxLoss, SSDConfig
    ctx = init_nncontext("ssd")
    torch.manual_seed(0)
    cfg = SSDConfig()
    ssd = SSD(num_classes=a.classes, cfg=cfg).to(ctx.device)
    crit = MultiBoxLoss(num_classes=a.classes)
    x = torch.randn(a.batch, 3, 300, 300, device=ctx.device)
    g = torch.Generator().manual_seed(1)
    targets = []
    for _ in range(a.batch):
        lo = torch.rand(2, 2, generator=g) * 0.5
        hi = lo + 0.2 + torch.rand(2, 2, generator=g) * 0.3
        lab = torch.randint(1, a.classes, (2, 1), generator=g).float()
        targets.append(torch.cat([lab, lo, hi.clamp(max=1.0)], 1).to(ctx.device))
    opt = torch.optim.SGD(ssd.parameters(), lr=1e-3, momentum=0.9)
    losses = []
    for _ in range(a.steps):
        loc, conf = ssd(x)
        loss = crit(loc, conf, ssd.priors, targets)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    print("multibox loss:", [round(v, 4) for v in losses])
    ssd.eval()
    with torch.no_grad():
        loc, conf = ssd(x)
        dets = DetectionOutputSSD(num_classes=a.classes, conf_thresh=0.01)(loc, conf, ssd.priors)
    print("detections per image:", [int(d.shape[0]) for d in dets])
    return losses


if __name__ == "__main__":
    main()
