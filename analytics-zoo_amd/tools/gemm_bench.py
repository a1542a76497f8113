#!/usr/bin/env python3
"""GEMM throughput: the zoo implicit-GEMM kernel used as a plain GEMM
(1x1 conv) vs torch.matmul (hipBLASLt) on the same bf16 shapes.

  python analytics-zoo_amd/tools/gemm_bench.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402

SHAPES = [  # (M, N, K): Y[M,N] = X[M,K] @ W[N,K]^T
    (4096, 4096, 4096), (8192, 8192, 8192), (802816, 64, 64), (802816, 256, 64), (802816, 64, 256),
    (200704, 512, 128), (200704, 128, 512), (50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512),
    (12544, 512, 2048),
]


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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=None, help="comma-separated indices into SHAPES")
    ap.add_argument("--zoo-only", action="store_true")
    ap.add_argument("--bert", action="store_true", help="BERT-base b128 x L128 linear-layer shapes")
    ap.add_argument("--tiles", default=None,
                    help="comma-separated igemm2 tiles to force (0 = auto; igemm2.hip I2Tile): per-tile time "
                         "and error of the plain 1x1-conv GEMM")
    a = ap.parse_args()
    shapes = SHAPES if a.shapes is None else [SHAPES[int(i)] for i in a.shapes.split(",")]
    if a.bert:  # (M, N, K) of QKV, attention output, FFN1, FFN2 at 16384 tokens
        shapes = [(16384, 2304, 768), (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072),
                  (4096, 2304, 768), (4096, 768, 3072)]
    dev = torch.device("cuda:0")
    if a.tiles:
        for M, N, K in shapes:
            x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
            x4 = x.view(1, M, 1, K)
            ref = x.float() @ w.float().t()
            rec = {"M": M, "N": N, "K": K}
            for t in [int(v) for v in a.tiles.split(",")]:
                C.igemm2_set(-1, t)
                fn = lambda: C.conv_fwd(x4, w, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1, None, None, None, 0, False, True, 0, 0,
                                        None, [], None, None, None, None, None)
                y = fn().view(M, N).float()
                rec["t%d_err" % t] = round(float((y - ref).abs().max() / ref.abs().max()), 5)
                tt = timeit(fn, 50)
                rec["t%d_us" % t] = round(tt * 1e6, 1)
                rec["t%d_TF" % t] = round(2.0 * M * N * K / tt / 1e12, 1)
            C.igemm2_set(-1, 0)
            print(json.dumps(rec), flush=True)
        return
    rows = []
    for M, N, K in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        x4 = x.view(1, M, 1, K)
        f = 2.0 * M * N * K
        t_z = timeit(lambda: C.conv_fwd(x4, w, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1, None, None, None, 0, False, True, 0, 0,
                                        None, [], None, None, None, None, None))
        st = torch.zeros(C.stat_len(N), device=dev)  # slotted statistics (as the BN path uses)
        t_zs = timeit(lambda: C.conv_fwd(x4, w, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1, None, None, st, 0, False, True, 0, 0,
                                         None, [], None, None, None, None, None))
        t_t = float("nan") if a.zoo_only else timeit(lambda: torch.matmul(x, w.t()))
        t_g = timeit(lambda: C.gemm(x, w, None, None, None, 0, False, True, None, None, None, None, None))
        err = float((C.gemm(x, w, None, None, None, 0, True, False, None, None, None, None, None) -
                     x.float() @ w.float().t()).abs().max() / (x.float() @ w.float().t()).abs().max())
        byts = 2.0 * (M * K + N * K + M * N)
        rows.append({"M": M, "N": N, "K": K, "gemm256_TF": round(f / t_g / 1e12, 1), "gemm256_err": err,
                     "zoo_TF": round(f / t_z / 1e12, 1), "torch_TF": round(f / t_t / 1e12, 1),
                     "zoo_us": round(t_z * 1e6, 1), "zoo_stats_us": round(t_zs * 1e6, 1), "torch_us": round(t_t * 1e6, 1),
                     "zoo_TBps": round(byts / t_z / 1e12, 2)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
