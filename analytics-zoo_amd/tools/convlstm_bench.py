#!/usr/bin/env python3
"""ConvLSTM2D / ConvLSTM3D forward+backward time: the one-launch-per-step path (_ConvLSTMFusedFn /
_ConvLSTM3DFusedFn, convlstm.hip), the 2-D whole-sequence path (_ConvLSTMSeqFn: recurrent conv +
step kernel forward, three launches per step backward) and the per-step loop (one recurrent conv +
one gate pass per step), and their agreement.

  python tools/convlstm_bench.py [--dims 2|3] [--T 32] [--batch 8] [--hw 32] [--cin 16] [--filters 32]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, default=32)
    ap.add_argument("--cin", type=int, default=16)
    ap.add_argument("--filters", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dims", type=int, default=2, choices=[2, 3])
    ap.add_argument("--modes", default=None, help="comma-separated subset of loop,seq,fused (profiling); "
                    "fused_np = fused with the persistent step kernels off, fused_rg = row-group persistent only, "
                    "fused_fks = forward K-split at every size, fused_ncp = gate-interleaved row-group forward epilogue (A/B)")
    a = ap.parse_args()
    from zoo.pipeline.api.keras.layers import recurrent as R
    torch.manual_seed(0)
    sp = (a.hw,) * a.dims
    if a.dims == 2:
        layer = R.ConvLSTM2D(a.filters, 3, 3, return_sequences=True, input_shape=(a.T, a.cin) + sp)
    else:
        layer = R.ConvLSTM3D(a.filters, 3, return_sequences=True, input_shape=(a.T, a.cin) + sp)
    layer._ensure_built((None, a.T, a.cin) + sp)
    layer = layer.cuda()
    x = torch.randn((a.batch, a.T, a.cin) + sp, device="cuda", requires_grad=True)
    res = {"bench": "convlstm%dd-fwd-bwd" % a.dims, "T": a.T, "batch": a.batch, "hw": a.hw, "cin": a.cin,
           "filters": a.filters}
    outs = {}
    names = {0: "loop", 1: "seq", 2: "fused", 3: "fused_np", 4: "fused_rg", 5: "fused_fks", 6: "fused_ncp"}
    from zoo.ops._kern import native
    # ConvLSTM3D has no separate whole-sequence mode: SEQ without FUSED is its per-step loop
    modes = (0, 1, 2) if a.dims == 2 else (0, 2)
    if a.modes:
        modes = [m for m in (0, 1, 2, 3, 4, 5, 6) if names[m] in a.modes.split(",") and (m != 1 or a.dims == 2)]
    for mode in modes:
        R._CONVLSTM_SEQ = mode > 0
        R._CONVLSTM_FUSED = mode >= 2
        native().convlstm_pers_set({3: 0, 4: 2, 5: 5, 6: 9}.get(mode, 1))

        def step():
            x.grad = None
            for p in layer.parameters():
                p.grad = None
            y = layer(x)
            y.float().square().mean().backward()
            return y
        for _ in range(2):
            y = step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            y = step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.iters * 1e3
        res["ms_%s" % names[mode]] = round(ms, 3)
        outs[mode] = (y.detach().float(), x.grad.detach().clone(), layer.Wh.grad.detach().clone())
    if "ms_loop" not in res:
        print(json.dumps(res), flush=True)
        return
    if "ms_seq" in res:
        res["speedup_seq"] = round(res["ms_loop"] / res["ms_seq"], 2)
    if "ms_fused" in res:
        res["speedup"] = round(res["ms_loop"] / res["ms_fused"], 2)
    for n in ("np", "rg", "fks", "ncp"):
        if "ms_fused_" + n in res:
            res["speedup_" + n] = round(res["ms_loop"] / res["ms_fused_" + n], 2)
    for mode in [m for m in (1, 2, 3, 4, 5, 6) if m in outs and 0 in outs]:
        for k, n in enumerate(("y", "dx", "dWh")):
            a0, a1 = outs[0][k], outs[mode][k]
            res["rel_%s_%s" % (names[mode], n)] = round(float((a0 - a1).abs().max() /
                                                              a0.abs().max().clamp_min(1e-12)), 5)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
