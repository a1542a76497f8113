#!/usr/bin/env python3
"""Correctness + speed check of the zoo conv kernels against PyTorch on one GPU.

For each ResNet-50 conv shape: forward / dgrad / wgrad through zoo._C are
compared with an fp32 PyTorch reference (relative max error), and timed
against torch's own bf16 channels_last conv (MIOpen) for context.

  python analytics-zoo_amd/tools/kernel_check.py [--batch 64] [--quick]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

import zoo._C as C

# (H, Cin, Cout, R, stride, pad) — every distinct ResNet-50 conv
RESNET50_CONVS = [
    (224, 4, 64, 7, 2, 3),     # stem (3 channels padded to 4)
    (56, 64, 64, 1, 1, 0),
    (56, 64, 64, 3, 1, 1),
    (56, 64, 256, 1, 1, 0),
    (56, 256, 64, 1, 1, 0),
    (56, 256, 128, 1, 1, 0),
    (56, 128, 128, 3, 2, 1),
    (28, 128, 512, 1, 1, 0),
    (56, 256, 512, 1, 2, 0),
    (28, 512, 128, 1, 1, 0),
    (28, 128, 128, 3, 1, 1),
    (28, 512, 256, 1, 1, 0),
    (28, 256, 256, 3, 2, 1),
    (14, 256, 1024, 1, 1, 0),
    (28, 512, 1024, 1, 2, 0),
    (14, 1024, 256, 1, 1, 0),
    (14, 256, 256, 3, 1, 1),
    (14, 1024, 512, 1, 1, 0),
    (14, 512, 512, 3, 2, 1),
    (7, 512, 2048, 1, 1, 0),
    (14, 1024, 2048, 1, 2, 0),
    (7, 2048, 512, 1, 1, 0),
    (7, 512, 512, 3, 1, 1),
]


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def check_one(N, H, Cin, Cout, R, st, pad, dev, do_time=True):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    w4 = (torch.randn(Cout, R, R, Cin, device=dev) / (R * R * Cin) ** 0.5).bfloat16()
    ktot = R * R * Cin
    ldb = (ktot + 7) // 8 * 8
    w2 = torch.zeros(Cout, ldb, device=dev, dtype=torch.bfloat16)
    w2[:, :ktot] = w4.reshape(Cout, ktot)
    # reference (fp32, NCHW)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w4.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pad)
    P = yr.shape[2]
    dy = torch.randn(N, P, P, Cout, device=dev).bfloat16()
    yr.backward(dy.float().permute(0, 3, 1, 2))
    res = {"shape": [N, H, Cin, Cout, R, st, pad]}

    stats = torch.zeros(2 * Cout, device=dev)
    y = C.conv_fwd(x, w2, R, R, st, st, pad, pad, 1, 1, 1, 1, None, None, stats, 0, False, True, 0, 0, None, [], None, None, None, None, None)
    yref = yr.detach().permute(0, 2, 3, 1)
    res["fwd_err"] = rel_err(y, yref)
    s_ref = torch.stack([y.float().sum((0, 1, 2)), (y.float() ** 2).sum((0, 1, 2))]).flatten()
    res["stats_err"] = rel_err(stats, s_ref)

    # dgrad: transposed conv with flipped weights
    wt = C.flip_weights(w4.reshape(Cout, -1).contiguous(), Cout, R, R, Cin, 0, 0, R, R, 1, 1)
    if Cin != 4:  # the stem's input never needs a gradient
        dx = C.conv_fwd(dy, wt, R, R, 1, 1, R - 1 - pad, R - 1 - pad, 1, 1, st, st, None, None, None, 0, False, True,
                        H, H, None, [], None, None, None, None, None)
        res["dgrad_err"] = rel_err(dx, xr.grad.permute(0, 2, 3, 1))
    dw = torch.zeros(Cout, ktot, device=dev)
    C.conv_wgrad(x, dy, dw, R, R, st, st, pad, pad, 1, 1)
    res["wgrad_err"] = rel_err(dw, wr.grad.permute(0, 2, 3, 1).reshape(Cout, ktot))

    if do_time:
        flops = 2.0 * N * P * P * Cout * ktot
        t_f = timeit(lambda: C.conv_fwd(x, w2, R, R, st, st, pad, pad, 1, 1, 1, 1, None, None, None, 0, False, True, 0, 0, None, [], None, None, None, None, None))
        t_d = timeit(lambda: C.conv_fwd(dy, wt, R, R, 1, 1, R - 1 - pad, R - 1 - pad, 1, 1, st, st, None, None, None, 0,
                                        False, True, H, H, None, [], None, None, None, None, None)) if Cin != 4 else float("nan")
        t_w = timeit(lambda: (dw.zero_(), C.conv_wgrad(x, dy, dw, R, R, st, st, pad, pad, 1, 1)))
        xt = x.permute(0, 3, 1, 2)  # channels_last view
        wt4 = w4.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        t_tf = timeit(lambda: F.conv2d(xt, wt4, stride=st, padding=pad))
        res.update({"zoo_fwd_ms": t_f, "zoo_dgrad_ms": t_d, "zoo_wgrad_ms": t_w, "torch_fwd_ms": t_tf,
                    "zoo_fwd_tflops": flops / t_f / 1e9, "zoo_dgrad_tflops": flops / t_d / 1e9,
                    "zoo_wgrad_tflops": flops / t_w / 1e9, "torch_fwd_tflops": flops / t_tf / 1e9})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = "cuda"
    rows = []
    shapes = RESNET50_CONVS[:4] if a.quick else RESNET50_CONVS
    for (H, ci, co, R, st, pad) in shapes:
        r = check_one(a.batch, H, ci, co, R, st, pad, dev)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
