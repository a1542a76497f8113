#!/usr/bin/env python3
"""Linear-layer weight gradient dW[N, K] (fp32) += dy[M, N]^T x[M, K] (bf16) at BERT-base
b128 x s128 shapes: hipBLASLt (fp32-out addmm beta=1, and bf16-out mm + add) vs the zoo
split-K wgrad kernel (csrc/kernels/wgrad.hip run as a 1x1 conv) and the 256x256-tile
LDS-DMA kernel (csrc/kernels/wgrad256.hip, ``zoo._C.linear_wgrad``).

  python analytics-zoo_amd/tools/wgrad_bench.py [--m 16384]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--more", action="store_true", help="also square / ResNet 1x1 shapes")
    ap.add_argument("--resnet", action="store_true", help="ResNet-50 b256 1x1 stride-1 conv shapes (M, Cout, Cin)")
    ap.add_argument("--conv", action="store_true",
                    help="ResNet-50 b256 3x3 / strided conv weight gradients through conv_wgrad (the route is "
                         "chosen by ZOO_WGRAD256_CONV_COUT: 0 = wgrad.hip, default 256 = implicit wgrad256)")
    a = ap.parse_args()
    if a.conv:
        return conv_main()
    dev = torch.device("cuda")
    M = a.m
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
    if a.more:
        shapes += [(4096, 4096), (1000, 2048), (256, 64), (64, 256), (512, 128), (2048, 512)]
    cases = [(M, N, K) for N, K in shapes]
    if a.resnet:
        cases = [(802816, 64, 64), (802816, 256, 64), (802816, 64, 256), (802816, 128, 256),
                 (200704, 512, 128), (200704, 128, 512), (200704, 256, 512), (50176, 1024, 256),
                 (50176, 256, 1024), (50176, 512, 1024), (12544, 2048, 512), (12544, 512, 2048)]
    for M, N, K in cases:
        dy = (torch.randn(M, N, device=dev) * 0.1).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        ref = (dy.float().t() @ x.float()).double()
        g = torch.zeros(N, K, device=dev)
        res = {"M": M, "N": N, "K": K}
        flop = 2.0 * M * N * K

        def lt_f32():
            torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32, beta=1, alpha=1, out=g)

        def lt_bf16():
            g.add_(torch.mm(dy.t(), x))

        def zoo():
            C.conv_wgrad(x.view(M, 1, 1, K), dy.view(M, 1, 1, N), g, 1, 1, 1, 1, 0, 0, 1, 1)

        def zoo256():
            C.linear_wgrad(dy, x, g)

        fns = (("hipblaslt_f32out", lt_f32), ("hipblaslt_bf16out_add", lt_bf16), ("zoo_wgrad", zoo),
               ("zoo_wgrad256", zoo256))
        if a.resnet:
            fns = fns[2:]
        for name, fn in fns:
            g.zero_()
            fn()
            torch.cuda.synchronize()
            err = ((g.double() - ref).norm() / ref.norm()).item()
            t = timeit(fn)
            res[name] = {"us": round(t * 1e6, 1), "tflops": round(flop / t / 1e12, 1), "rel_err": float("%.2e" % err)}
        print(json.dumps(res), flush=True)


def conv_main():
    dev = torch.device("cuda")
    # (N, H, Cin, Cout, R, stride, pad, count in the network)
    cases = [(256, 56, 64, 64, 3, 1, 1, 3), (256, 56, 128, 128, 3, 2, 1, 1), (256, 28, 128, 128, 3, 1, 1, 3),
             (256, 28, 256, 256, 3, 2, 1, 1), (256, 14, 256, 256, 3, 1, 1, 5), (256, 14, 512, 512, 3, 2, 1, 1),
             (256, 7, 512, 512, 3, 1, 1, 2), (256, 56, 256, 512, 1, 2, 0, 1), (256, 28, 512, 1024, 1, 2, 0, 1),
             (256, 14, 1024, 2048, 1, 2, 0, 1)]
    total = 0.0
    for N, H, Cin, Cout, R, st, pad, cnt in cases:
        x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = (torch.randn(N, P, P, Cout, device=dev) * 0.1).bfloat16()
        g = torch.zeros(Cout, R * R * Cin, device=dev)

        def fn():
            C.conv_wgrad(x, dy, g, R, R, st, st, pad, pad, 1, 1)
        t = timeit(fn)
        flop = 2.0 * N * P * P * Cout * R * R * Cin
        total += t * cnt
        print(json.dumps({"N": N, "H": H, "Cin": Cin, "Cout": Cout, "R": R, "stride": st, "count": cnt,
                          "us": round(t * 1e6, 1), "tflops": round(flop / t / 1e12, 1),
                          "route_cout": os.environ.get("ZOO_WGRAD256_CONV_COUT", "256")}), flush=True)
        del x, dy, g
    print(json.dumps({"network_ms": round(total * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
