#!/usr/bin/env python3
"""A/B of the implicit-GEMM conv kernels on one MI355X, in ONE process with interleaved
rounds (cdna_hip_programming.md §5.4 rule 24):

  * igemm (csrc/kernels/igemm.hip, 128x{64,128} tiles)            -> mode 0
  * igemm2 (csrc/kernels/igemm2.hip, large tiles, 3-stage ring)   -> mode 1, per tile config

over the ResNet-50 b256 conv shapes (forward and data-gradient) and the transformer GEMMs,
checking igemm2 against igemm (bf16 outputs, BN statistics) and, for the GEMMs, timing
hipBLASLt (torch.mm) on the same operands.

  python analytics-zoo_amd/tools/igemm2_bench.py [--batch 256] [--tiles 0,1,2,3,4,5,6,7] [--quick]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402
from zoo.ops import _kern  # noqa: E402
from tools.kernel_check import RESNET50_CONVS  # noqa: E402

COUNTS = [1, 1, 3, 4, 2, 1, 1, 4, 1, 3, 3, 1, 1, 6, 1, 5, 5, 1, 1, 3, 1, 2, 2]
TILE_NAMES = {0: "auto", 1: "128x128", 2: "256x128", 3: "256x128s3", 4: "256x64", 5: "256x256",
              6: "128x64s3", 7: "128x128s3"}


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def time_fns(fns, rounds=5, iters=10):
    """fns: {name: fn}. Interleaved rounds; returns {name: median ms}."""
    res = {k: [] for k in fns}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                f()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) / iters)
    return {k: sorted(v)[len(v) // 2] for k, v in res.items()}


def with_mode(mode, tile, fn):
    def run():
        C.igemm2_set(mode, tile)
        return fn()
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tiles", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--no-gemm", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    rows = []
    tot = {}
    shapes = list(zip(RESNET50_CONVS, COUNTS))
    if a.quick:
        shapes = [s for s in shapes if s[0][0] in (56, 14)][:6]
    for (H, Cin, Cout, R, st, pad), cnt in shapes:
        if Cin % 64:
            continue
        N = a.batch
        x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
        ktot = R * R * Cin
        w2 = (torch.randn(Cout, ktot, device=dev) / math.sqrt(ktot)).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, Cout, device=dev).bfloat16()
        flops = 2.0 * N * P * P * Cout * ktot
        for op in ("fwd", "dgrad"):
            if op == "dgrad" and Cout % 64:
                continue
            # as in the model: slotted statistics (stat_len) for the forward; the data gradient with
            # the producer's fused BN-backward (ReLU mask z, pre-BN y, mean / inv, sums)
            stats = torch.zeros(C.stat_len(Cout) if op == "fwd" else C.stat_len(Cin), device=dev)
            yprod = torch.randn(N, H, H, Cin, device=dev).bfloat16()
            zprod = torch.relu(yprod)
            mean = torch.zeros(Cin, device=dev)
            inv = torch.ones(Cin, device=dev)

            def fwd():
                stats.zero_()
                return _kern.conv_fwd(x, w2, R, R, (st, st), (pad, pad), stats=stats)

            def dgrad():
                stats.zero_()
                return _kern.conv_dgrad(dy, w2, Cout, R, R, Cin, H, H, (st, st), (pad, pad),
                                        bstats=(zprod, yprod, mean, inv, stats))
            fn = fwd if op == "fwd" else dgrad
            C.igemm2_set(0, 0)
            ref = fn().clone()
            ref_stats = stats.clone()
            fns = {"igemm": with_mode(0, 0, fn)}
            row = {"shape": [H, Cin, Cout, R, st, pad], "op": op, "n": cnt}
            for t in tiles:
                C.igemm2_set(1, t)
                out = fn()
                torch.cuda.synchronize()
                e = rel(out, ref)
                row["err_" + TILE_NAMES[t]] = round(e, 5)
                row["serr_" + TILE_NAMES[t]] = round(rel(stats[:2 * (Cout if op == "fwd" else Cin)],
                                                         ref_stats[:2 * (Cout if op == "fwd" else Cin)]), 6)
                fns[TILE_NAMES[t]] = with_mode(1, t, fn)
            ms = time_fns(fns)
            for k, v in ms.items():
                row["ms_" + k] = round(v, 4)
                row["tf_" + k] = round(flops / v / 1e9, 1)
                tot.setdefault(op + "_" + k, 0.0)
                tot[op + "_" + k] += v * cnt
            rows.append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps({"whole_network_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)
    if not a.no_gemm:
        gemms = [(16384, 768, 768), (16384, 768, 2304), (16384, 768, 3072), (16384, 3072, 768), (4096, 4096, 4096),
                 (8192, 8192, 8192)]
        for (M, K, Nn) in gemms:
            x = torch.randn(M, 1, 1, K, device=dev).bfloat16()
            w = (torch.randn(Nn, K, device=dev) / math.sqrt(K)).bfloat16()
            fn = lambda: _kern.conv_fwd(x, w, 1, 1)  # noqa: E731
            C.igemm2_set(0, 0)
            ref = fn().clone()
            fns = {"igemm": with_mode(0, 0, fn), "hipblaslt": lambda: torch.mm(x.view(M, K), w.t())}
            row = {"gemm": [M, Nn, K]}
            for t in tiles:
                C.igemm2_set(1, t)
                row["err_" + TILE_NAMES[t]] = round(rel(fn(), ref), 5)
                fns[TILE_NAMES[t]] = with_mode(1, t, fn)
            ms = time_fns(fns)
            for k, v in ms.items():
                row["tf_" + k] = round(2.0 * M * Nn * K / v / 1e9, 1)
            rows.append(row)
            print(json.dumps(row), flush=True)
    C.igemm2_set(1, 0)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
