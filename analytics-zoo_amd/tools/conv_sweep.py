#!/usr/bin/env python3
"""Whole-network conv time of ResNet-50 (batch N, bf16 NHWC) per op, weighted by
how often each conv shape occurs: one number per op for A/B-ing kernel knobs
(env vars such as ZOO_IGEMM_BN) on the GPU.

  python analytics-zoo_amd/tools/conv_sweep.py [--batch 256] [--ops fwd,dgrad,wgrad] [--detail]
      [--roofline out.md]

--roofline writes a per-conv table: time, FLOP, TF/s and the minimum HBM bytes of each op
(operands read once, result written once: fwd reads x + w and writes y in bf16, dgrad reads
dy + w and writes dx, wgrad reads x + dy and writes the fp32 dW), each as a percentage of
its bound -- the MFMA bound at 2.5 PF/s dense bf16 or the HBM bound at 8 TB/s, whichever is
larger ("%SOL" = bound time / measured time).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zoo._C as C  # noqa: E402
from zoo.ops import _kern  # noqa: E402
from tools.kernel_check import RESNET50_CONVS  # noqa: E402

# occurrences of each RESNET50_CONVS shape in ResNet-50 v1.5 (53 convs)
COUNTS = [1, 1, 3, 4, 2, 1, 1, 4, 1, 3, 3, 1, 1, 6, 1, 5, 5, 1, 1, 3, 1, 2, 2]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--detail", action="store_true")
    ap.add_argument("--roofline", default=None)
    a = ap.parse_args()
    roof = []
    ops = a.ops.split(",")
    dev = torch.device("cuda")
    tot = {o: 0.0 for o in ops}
    assert len(COUNTS) == len(RESNET50_CONVS)
    for (H, Cin, Cout, R, st, pad), cnt in zip(RESNET50_CONVS, COUNTS):
        N = a.batch
        x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
        ktot = R * R * Cin
        w2 = torch.zeros(Cout, (ktot + 7) // 8 * 8, device=dev, dtype=torch.bfloat16)
        w2[:, :ktot] = (torch.randn(Cout, ktot, device=dev) / ktot ** 0.5).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, Cout, device=dev).bfloat16()
        stats = torch.zeros(C.stat_len(Cout), device=dev)
        row = {"shape": [H, Cin, Cout, R, st, pad], "n": cnt}
        if "fwd" in ops:
            row["fwd"] = timeit(lambda: _kern.conv_fwd(x, w2, R, R, (st, st), (pad, pad), stats=stats))
        if "dgrad" in ops and Cin != 4:
            row["dgrad"] = timeit(lambda: _kern.conv_dgrad(dy, w2, Cout, R, R, Cin, H, H, (st, st), (pad, pad)))
        if "wgrad" in ops:
            dw = torch.zeros(Cout, ktot, device=dev)
            row["wgrad"] = timeit(lambda: C.conv_wgrad(x, dy, dw, R, R, st, st, pad, pad, 1, 1))
            if R == 1 and st == 1:  # library GEMM for comparison: dW = dY^T X, fp32 output
                x2, dy2 = x.reshape(-1, Cin), dy.reshape(-1, Cout)
                row["wgrad_blas"] = timeit(lambda: torch.mm(dy2.t(), x2, out_dtype=torch.float32))
        if "fwd" in ops and R == 1 and st == 1:
            x2 = x.reshape(-1, Cin)
            row["fwd_blas"] = timeit(lambda: torch.mm(x2, w2[:, :Cin].t()))
        if "dgrad" in ops and R == 1 and st == 1:
            dy2 = dy.reshape(-1, Cout)
            wt = w2[:, :Cin].contiguous()
            row["dgrad_blas"] = timeit(lambda: torch.mm(dy2, wt))
        for o in ops:
            tot[o] += row.get(o, 0.0) * cnt
            if o in row:
                roof.append(_roof_row(o, N, H, Cin, Cout, R, st, P, cnt, row[o]))
        if a.detail:
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
        del x, dy, w2
    print(json.dumps({"batch": a.batch, "ms_per_step": {o: round(v, 3) for o, v in tot.items()},
                      "knobs": {k: v for k, v in os.environ.items() if k.startswith("ZOO_")}}), flush=True)
    if a.roofline:
        _write_roofline(a.roofline, a.batch, roof, tot)


PEAK_TFLOPS, HBM_TBS = 2500.0, 8.0


def _roof_row(op, N, H, Cin, Cout, R, st, P, cnt, ms):
    flop = 2.0 * N * P * P * Cout * Cin * R * R
    x, y, w = N * H * H * Cin * 2, N * P * P * Cout * 2, Cout * Cin * R * R * 2
    byt = {"fwd": x + w + y, "dgrad": y + w + x, "wgrad": x + y + 2 * w}[op]
    t_mfma = flop / (PEAK_TFLOPS * 1e12) * 1e3
    t_hbm = byt / (HBM_TBS * 1e12) * 1e3
    bound = "MFMA" if t_mfma >= t_hbm else "HBM"
    return {"op": op, "shape": f"{H}x{H} {Cin}->{Cout} {R}x{R}/s{st}", "n": cnt, "ms": ms,
            "tflops": flop / ms / 1e9, "gbytes": byt / 1e9, "tbs": byt / ms / 1e9, "bound": bound,
            "sol": max(t_mfma, t_hbm) / ms}


def _write_roofline(path, batch, roof, tot):
    lines = [f"# ResNet-50 per-conv roofline, batch {batch} (tools/conv_sweep.py --roofline)", "",
             f"Bounds: MFMA {PEAK_TFLOPS:.0f} TF/s dense bf16, HBM {HBM_TBS:.0f} TB/s; min bytes = operands "
             "read once + result written once. %SOL = bound time / measured time.", "",
             "| op | conv (input, Cin->Cout, kernel/stride) | n | ms each | ms x n | TF/s | GB | TB/s | bound | %SOL |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r in sorted(roof, key=lambda r: -r["ms"] * r["n"]):
        lines.append(f"| {r['op']} | {r['shape']} | {r['n']} | {r['ms']:.3f} | {r['ms'] * r['n']:.3f} | "
                     f"{r['tflops']:.0f} | {r['gbytes']:.3f} | {r['tbs']:.2f} | {r['bound']} | {100 * r['sol']:.0f}% |")
    lines += ["", "Totals (ms per training step, convs only): " +
              ", ".join(f"{o} {v:.3f}" for o, v in tot.items())]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
