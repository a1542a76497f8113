#!/usr/bin/env python3
"""Isolate the one-launch ConvLSTM step kernels (csrc/kernels/convlstm.hip) for profiling:
whole-sequence forward / backward at the ConvLSTM2D bench shape, plus the forward with no
recurrent operand (X = None: the cell epilogue alone). Run under rocprofv3 --kernel-trace --stats.

  python tools/convlstm_step_bench.py [--T 32] [--batch 8] [--hw 32] [--filters 32] [--iters 10]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, default=32)
    ap.add_argument("--filters", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from zoo.ops._native import native
    C_ = native()
    dev = torch.device("cuda")
    T, B, H, W, f = a.T, a.batch, a.hw, a.hw, a.filters
    K = 4 * f
    cph = (f + 7) // 8 * 8
    M = B * H * W
    torch.manual_seed(0)
    wt = (torch.randn(K, 9 * cph, device=dev) * 0.05).to(torch.bfloat16)
    wf = (torch.randn(cph, 9 * K, device=dev) * 0.05).to(torch.bfloat16)
    gxs = torch.randn(T, M, K, device=dev) * 0.5
    hist = torch.zeros(T + 1, B, H, W, cph, dtype=torch.bfloat16, device=dev)
    hseq = torch.empty(T, M, f, device=dev)
    cseq = torch.empty_like(hseq)
    acts = torch.empty(T, M, K, device=dev)
    dout = torch.randn(T, M, f, device=dev)
    dc = torch.empty(M, f, device=dev)
    dgxs = torch.empty(T, M, K, device=dev)
    dgb = torch.zeros(T, B, H, W, K, dtype=torch.bfloat16, device=dev)
    for _ in range(a.iters):
        C_.convlstm_fwd_seq(gxs, wt, B, 1, H, W, 1, 3, 3, hist, hseq, cseq, acts, 2, 1)
        C_.convlstm_bwd_seq(dout, True, wf, B, 1, H, W, 1, 3, 3, acts, cseq, dc, dgxs, dgb, 2, 1)
        for s in range(T):    # epilogue only (no recurrent GEMM)
            C_.convlstm_fwd_step(None, wt, B, 1, H, W, 1, 3, 3, gxs[s], None, hseq[s], cseq[s], acts[s],
                                 hist[s + 1], 2, 1)
    torch.cuda.synchronize()
    print("done", float(hseq.abs().mean()), float(dgxs.abs().mean()), flush=True)


if __name__ == "__main__":
    main()
