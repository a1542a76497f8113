#!/usr/bin/env python3
"""Per-conv roofline of the ResNet-50 (b256, bf16 NHWC) 1x1 convolutions with the epilogues the
training step actually runs:

  fwd   : conv + BatchNorm statistics (EPI 1)
  dgrad : data gradient + fused BN-backward of the producing unit (EPI 2): ReLU mask recomputed
          from y (zmode 1, conv3 / downsample-style) or a 1-bit mask + residual-gradient add
          (zmode 2, conv1 of identity blocks)

For each call: time (median of interleaved rounds), FLOP, the minimum HBM bytes (every operand
read once, every output written once) and the percentage of the MFMA (2.5 PF bf16 dense) and
HBM (8 TB/s) bounds reached. ``--ab`` times the streaming 1x1 kernel (pw.hip) against the
igemm / igemm2 route in the same process.

  python analytics-zoo_amd/tools/pw_bench.py [--batch 256] [--ab] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PEAK_TF = 2500.0
PEAK_TBS = 8.0

# (spatial H, Cin, Cout, count) of every stride-1 1x1 conv in ResNet-50 v1.5
SHAPES = [
    (56, 64, 64, 1), (56, 64, 256, 4), (56, 256, 64, 2), (56, 256, 128, 1),
    (28, 128, 512, 4), (28, 512, 128, 3), (28, 512, 256, 1),
    (14, 256, 1024, 6), (14, 1024, 256, 5), (14, 1024, 512, 1),
    (7, 512, 2048, 3), (7, 2048, 512, 2),
]


def _ev_time(fn, rounds=7, iters=5):
    ts = []
    for _ in range(2):
        fn()
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    ts.sort()
    return ts[len(ts) // 2] * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ab", action="store_true")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from zoo.ops import _kern
    from zoo.ops._native import native
    C = native()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    rows = []
    modes = [("pw", 1), ("ref", 0)] if a.ab else [("cur", -1)]
    for (H, Cin, Cout, cnt) in SHAPES:
        N = a.batch
        M = N * H * H
        x = (torch.randn(N, H, H, Cin, device=dev, generator=g)).bfloat16()
        w = (torch.randn(Cout, Cin, device=dev, generator=g) / Cin ** 0.5).bfloat16()
        dy = torch.randn(N, H, H, Cout, device=dev, generator=g).bfloat16()
        # the producing unit of x (for the dgrad epilogue): its raw output y and BN constants
        yprod = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
        mean = torch.randn(Cin, device=dev, generator=g) * 0.1
        inv = torch.rand(Cin, device=dev, generator=g) + 0.5
        gam = torch.rand(Cin, device=dev, generator=g) + 0.5
        bet = torch.randn(Cin, device=dev, generator=g) * 0.1
        mask = torch.randint(0, 256, (M * Cin // 8,), device=dev, generator=g, dtype=torch.uint8)
        resid = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
        stats = torch.zeros(C.stat_len(Cout), device=dev)
        sums = torch.zeros(C.stat_len(Cin), device=dev)
        flop = 2.0 * M * Cin * Cout
        cases = {
            "fwd": (lambda: _kern.conv_fwd(x, w, 1, 1, stats=stats),
                    2.0 * M * (Cin + Cout) + 2.0 * Cin * Cout),
            "dgrad_z1": (lambda: _kern.conv_dgrad(dy, w, Cout, 1, 1, Cin, H, H,
                                                  bstats=(None, yprod, mean, inv, sums, gam, bet)),
                         2.0 * M * (Cout + 2 * Cin) + 2.0 * Cin * Cout),
            "dgrad_z2r": (lambda: _kern.conv_dgrad(dy, w, Cout, 1, 1, Cin, H, H, resid=resid,
                                                   bstats=(mask, yprod, mean, inv, sums)),
                          2.0 * M * (Cout + 3 * Cin) + M * Cin / 8.0 + 2.0 * Cin * Cout),
        }
        for name, (fn, by) in cases.items():
            row = {"shape": [H, Cin, Cout], "n": cnt, "op": name, "GFLOP": round(flop / 1e9, 2),
                   "MB": round(by / 1e6, 1)}
            for lab, mode in modes:
                if mode >= 0:
                    C.pw_set(mode)
                us = _ev_time(fn)
                row[lab + "_us"] = round(us, 1)
                row[lab + "_pct_mfma"] = round(100 * flop / (us * 1e-6) / (PEAK_TF * 1e12), 1)
                row[lab + "_pct_hbm"] = round(100 * by / (us * 1e-6) / (PEAK_TBS * 1e12), 1)
            rows.append(row)
            print(json.dumps(row), flush=True)
        del x, w, dy, yprod, resid, mask
    if a.ab:
        C.pw_set(-1)
    tot = {}
    for r in rows:
        for k, v in r.items():
            if k.endswith("_us"):
                key = r["op"] + ":" + k[:-3]
                tot[key] = tot.get(key, 0.0) + v * r["n"] / 1e3
    print(json.dumps({"batch": a.batch, "weighted_ms": {k: round(v, 3) for k, v in sorted(tot.items())}}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "weighted_ms": tot}, f, indent=1)


if __name__ == "__main__":
    main()
