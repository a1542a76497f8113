#!/usr/bin/env python3
"""Bandwidth of the BN apply kernels on the ResNet-50 b256 activation shapes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402

SHAPES = [(802816, 64), (802816, 256), (200704, 128), (200704, 512), (50176, 256), (50176, 1024), (12544, 512),
          (12544, 2048)]


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    dev = torch.device("cuda:0")
    for M, Cc in SHAPES:
        x = torch.randn(M, Cc, device=dev).bfloat16()
        r = torch.randn(M, Cc, device=dev).bfloat16()
        stats = torch.cat([x.float().sum(0), (x.float() ** 2).sum(0)])
        g = torch.ones(Cc, device=dev)
        b = torch.zeros(Cc, device=dev)
        rm, rv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
        sm, si = torch.empty(Cc, device=dev), torch.empty(Cc, device=dev)
        t_f = timeit(lambda: C.bn_fwd_apply(x, stats, g, b, None, rm, rv, sm, si, 1e-5, 0.1, True, True))
        t_fr = timeit(lambda: C.bn_fwd_apply(x, stats, g, b, r, rm, rv, sm, si, 1e-5, 0.1, True, True))
        sums = torch.randn(2 * Cc, device=dev)
        dg, db = torch.zeros(Cc, device=dev), torch.zeros(Cc, device=dev)
        t_b = timeit(lambda: C.bn_bwd_apply(x, r, x, sm, si, g, sums, False, dg, db))
        t_ref = timeit(lambda: torch.add(x, r))
        byt = M * Cc * 2
        print(json.dumps({"M": M, "C": Cc, "fwd_TBps": round(2 * byt / t_f / 1e12, 2),
                          "fwd_resid_TBps": round(3 * byt / t_fr / 1e12, 2),
                          "bwd_TBps": round(4 * byt / t_b / 1e12, 2), "torch_add_TBps": round(3 * byt / t_ref / 1e12, 2),
                          "fwd_us": round(t_f * 1e6, 1), "bwd_us": round(t_b * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
