#!/usr/bin/env python3
"""Where a static int8 ResNet-50 loses agreement with its bf16 model: per residual block, the cosine
between the bf16 block output and the dequantised int8 block output (each fed its own chain), plus
per-channel range statistics of the calibration activations.
  python tools/quant_diag.py [--steps 80] [--lr 0.05] [--hw 224] [--clip 0]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--clip", type=float, default=0.0)
    ap.add_argument("--scales", default="channel")
    a = ap.parse_args()
    from zoo.models.image.resnet import resnet50
    from zoo.ops.qresnet import Int8ResNet, quantize_act
    from zoo.utils.synthetic import class_templates, sample, train_briefly
    T = class_templates(16, a.hw, device="cuda")
    torch.manual_seed(0)
    m = resnet50(num_classes=16).cuda()
    acc = train_briefly(m, T, steps=a.steps, lr=a.lr)
    cal, _ = sample(T, 64, seed=11)
    xt, _ = sample(T, 64, seed=12)
    q = Int8ResNet(m, cal, act_scales=a.scales, act_clip=a.clip)
    rows = []
    with torch.no_grad():
        h = q._stem(xt)
        xq = quantize_act(h, q.s_in, q.fmt)
        hb = h
        for i, (blk, u) in enumerate(q.blocks):
            s_x, s_sc, s_o = blk._q_scales
            sc = u["down"](xq) if "down" in u else xq
            h1 = u["conv1"](xq)
            xq = u["conv3"](u["conv2"](h1), resid=sc, s_resid=s_sc)
            scb = blk.down(hb) if blk.down is not None else hb
            hb = blk.conv3(blk.conv2(blk.conv1(hb)), resid=scb)
            so = s_o if torch.is_tensor(s_o) else torch.tensor(s_o, device=xq.device)
            deq = xq.float() * so
            ref = hb.float()
            cos = F.cosine_similarity(deq.flatten(), ref.flatten(), dim=0).item()
            ch = ref.abs().reshape(-1, ref.shape[-1])
            amax = ch.amax(0)
            p999 = ch.kthvalue(max(1, int(ch.shape[0] * 0.999)), dim=0).values
            rows.append({"block": i, "cos": round(cos, 5),
                         "chan_amax_max_over_median": round(float(amax.max() / amax.median().clamp_min(1e-9)), 2),
                         "median_amax_over_p999": round(float((amax / p999.clamp_min(1e-9)).median()), 2),
                         "dead_channels": int((amax == 0).sum())})
    print(json.dumps({"task_acc": acc, "scales": a.scales, "clip": a.clip, "blocks": rows}))


if __name__ == "__main__":
    main()
