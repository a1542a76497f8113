#!/usr/bin/env python3
"""Run ONE conv / GEMM kernel configuration back to back (for rocprofv3 PMC passes).

  python igemm2_one.py --gemm 8192,8192,8192 --tile 5 [--iters 20] [--old]
  python igemm2_one.py --conv 14,256,256,3,1,1 --tile 5 [--batch 256] [--dgrad]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402
from zoo.ops import _kern  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", default=None)
    ap.add_argument("--conv", default=None)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--old", action="store_true", help="igemm.hip instead of igemm2.hip")
    ap.add_argument("--gemm256", action="store_true", help="gemm256.hip (plain GEMMs only)")
    ap.add_argument("--dgrad", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    C.igemm2_set(0 if a.old else 1, a.tile)
    if a.gemm:
        M, N, K = [int(v) for v in a.gemm.split(",")]
        x = (torch.rand(M, 1, 1, K, device=dev) * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / math.sqrt(K)).bfloat16()
        if a.gemm256:
            fn = lambda: C.gemm(x.view(M, K), w, None, None, None, 0, False, True, None, None, None, None, None)  # noqa: E731
        else:
            fn = lambda: _kern.conv_fwd(x, w, 1, 1)  # noqa: E731
    else:
        H, Cin, Cout, R, st, pad = [int(v) for v in a.conv.split(",")]
        N = a.batch
        x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
        w = (torch.randn(Cout, R * R * Cin, device=dev) / math.sqrt(R * R * Cin)).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, Cout, device=dev).bfloat16()
        stats = torch.zeros(C.stat_len(Cout), device=dev)
        if a.dgrad:
            fn = lambda: _kern.conv_dgrad(dy, w, Cout, R, R, Cin, H, H, (st, st), (pad, pad))  # noqa: E731
        else:
            fn = lambda: _kern.conv_fwd(x, w, R, R, (st, st), (pad, pad), stats=stats)  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
