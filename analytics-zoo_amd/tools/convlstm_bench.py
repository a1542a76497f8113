#!/usr/bin/env python3
"""ConvLSTM2D forward+backward time: the one-launch-per-step path (_ConvLSTMFusedFn,
convlstm.hip), the whole-sequence path (_ConvLSTMSeqFn: recurrent conv + step kernel forward,
three launches per step backward) and the per-step autograd loop, and their agreement.

  python tools/convlstm_bench.py [--T 32] [--batch 8] [--hw 32] [--cin 16] [--filters 32]"""
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
    a = ap.parse_args()
    from zoo.pipeline.api.keras.layers import recurrent as R
    torch.manual_seed(0)
    layer = R.ConvLSTM2D(a.filters, 3, 3, return_sequences=True, input_shape=(a.T, a.cin, a.hw, a.hw))
    layer._ensure_built((None, a.T, a.cin, a.hw, a.hw))
    layer = layer.cuda()
    x = torch.randn(a.batch, a.T, a.cin, a.hw, a.hw, device="cuda", requires_grad=True)
    res = {"bench": "convlstm2d-fwd-bwd", "T": a.T, "batch": a.batch, "hw": a.hw, "cin": a.cin,
           "filters": a.filters}
    outs = {}
    names = {0: "loop", 1: "seq", 2: "fused"}
    for mode in (0, 1, 2):
        R._CONVLSTM_SEQ = mode > 0
        R._CONVLSTM_FUSED = mode == 2

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
    res["speedup_seq"] = round(res["ms_loop"] / res["ms_seq"], 2)
    res["speedup"] = round(res["ms_loop"] / res["ms_fused"], 2)
    for mode in (1, 2):
        for k, n in enumerate(("y", "dx", "dWh")):
            a0, a1 = outs[0][k], outs[mode][k]
            res["rel_%s_%s" % (names[mode], n)] = round(float((a0 - a1).abs().max() /
                                                              a0.abs().max().clamp_min(1e-12)), 5)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
