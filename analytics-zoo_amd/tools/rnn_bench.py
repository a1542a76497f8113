#!/usr/bin/env python3
"""LSTM/GRU layer timing: persistent HIP kernel (zoo.ops.rnn) vs the per-step
path (one MFMA GEMM + elementwise ops per time step). Forward+backward, fp32
activations, bf16 MFMA. Usage: rnn_bench.py [B] [T] [D]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from zoo.pipeline.api.keras import layers as L  # noqa: E402


def run(layer, x, fused, iters=10):
    layer._fused_ok = (lambda x_: type(layer)._fused_ok(layer, x_)) if fused else (lambda x_: False)
    for _ in range(3):
        layer(x).sum().backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        layer(x).sum().backward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    D = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    for name in ("LSTM", "GRU"):
        for H in (64, 128, 256):
            layer = getattr(L, name)(H, return_sequences=True, input_shape=(T, D))
            layer._ensure_built((None, T, D))
            layer = layer.cuda()
            x = torch.randn(B, T, D, device="cuda", requires_grad=True)
            tf = run(layer, x, True)
            ts = run(layer, x, False)
            print("%-4s B=%d T=%d D=%d H=%3d  fused %.3f ms  per-step %.3f ms  speedup %.1fx" % (name, B, T, D, H, tf,
                                                                                               ts, ts / tf),
                  flush=True)


if __name__ == "__main__":
    main()
