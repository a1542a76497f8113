#!/usr/bin/env python3
"""Probe the memory-bound 1x1 convolutions of ResNet-50 (b256): one launch per
variant, run under ``rocprofv3 --kernel-trace --stats`` to read exact kernel
times, plus a streaming-copy reference of the same bytes (HBM roofline).

  python tools/conv1x1_probe.py [--shape 56,64,256] [--iters 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402
from zoo.ops import _kern  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="56,64,256;56,256,64;28,128,512;14,256,1024;14,1024,256;7,2048,512;28,128,128")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for sh in a.shapes.split(";"):
        H, Cin, Cout = (int(v) for v in sh.split(","))
        N = a.batch
        x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
        w = (torch.randn(Cout, Cin, device=dev) / Cin ** 0.5).bfloat16()
        dy = torch.randn(N, H, H, Cout, device=dev).bfloat16()
        stats = torch.zeros(C.stat_len(Cout), device=dev)
        M = N * H * H
        byt = (M * Cin + M * Cout + Cin * Cout) * 2
        flops = 2.0 * M * Cin * Cout
        r = {}
        r["fwd+stats"] = timeit(lambda: _kern.conv_fwd(x, w, 1, 1, stats=stats), a.iters)
        r["fwd"] = timeit(lambda: _kern.conv_fwd(x, w, 1, 1), a.iters)
        r["dgrad"] = timeit(lambda: _kern.conv_dgrad(dy, w, Cout, 1, 1, Cin, H, H), a.iters)
        src = torch.empty(byt // 8, device=dev, dtype=torch.float32)  # read byt/2 + write byt/2
        dst = torch.empty_like(src)
        r["copy_same_bytes"] = timeit(lambda: dst.copy_(src), a.iters)
        print("shape %-14s M=%d  min bytes %.0f MB  %.1f GFLOP" % (sh, M, byt / 1e6, flops / 1e9))
        for k, us in r.items():
            print("   %-16s %8.1f us  %6.2f TB/s  %6.0f TF/s" % (k, us, byt / us / 1e6, flops / us / 1e6))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
