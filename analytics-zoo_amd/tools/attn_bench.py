"""Fused attention throughput (TFLOP/s) on BERT / long-sequence shapes.

python tools/attn_bench.py [--iters 20]
fwd FLOPs = 4*B*H*L*S*D (halved when causal); bwd = 2.5x fwd (dK/dV + dQ
passes recompute S, so the kernels execute 3.5x fwd MFMA work).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from zoo.ops._native import native  # noqa: E402

SHAPES = [  # B, H, L, D, causal
    (32, 12, 512, 64, False),   # BERT-base, seq 512
    (16, 16, 1024, 64, True),
    (8, 16, 2048, 128, False),
    (8, 16, 2048, 128, True),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bert", action="store_true",
                    help="BERT-base training shape (B 128, H 12, L 128, D 64, key mask) with / without "
                         "probability dropout and at half / quarter batch: is the pass latency- or work-bound?")
    a = ap.parse_args()
    C = native()
    if a.bert:
        for B in (128, 64, 32):
            for p in (0.0, 0.1):
                q, k, v = (torch.randn(B, 12, 128, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
                mask = torch.zeros(B, 128, device="cuda")
                mask[:, 100:] = -10000.0
                o, lse = C.attn_fwd(q, k, v, mask, False, p, 7)
                do = torch.randn_like(o)
                tf = timeit(lambda: C.attn_fwd(q, k, v, mask, False, p, 7), a.iters)
                tb = timeit(lambda: C.attn_bwd(do, q, k, v, mask, o, lse, False, p, 7), a.iters)
                fl = 4.0 * B * 12 * 128 * 128 * 64
                print("BERT B%d pdrop %.1f  fwd %.1f us %.0f TF | bwd %.1f us %.0f TF" %
                      (B, p, tf * 1e3, fl / tf / 1e9, tb * 1e3, 2.5 * fl / tb / 1e9), flush=True)
        return
    for B, H, L, D, causal in SHAPES:
        q, k, v = (torch.randn(B, H, L, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        o, lse = C.attn_fwd(q, k, v, None, causal)
        do = torch.randn_like(o)
        tf = timeit(lambda: C.attn_fwd(q, k, v, None, causal), a.iters)
        tb = timeit(lambda: C.attn_bwd(do, q, k, v, None, o, lse, causal), a.iters)
        fl = 4.0 * B * H * L * L * D * (0.5 if causal else 1.0)
        # torch SDPA for comparison (math/flash backend chosen by torch)
        qs, ks, vs = (t.clone().requires_grad_(True) for t in (q, k, v))
        tt = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=causal), a.iters)
        ot = torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=causal)
        ttb = timeit(lambda: torch.autograd.grad(ot, (qs, ks, vs), do, retain_graph=True), a.iters)
        print("B%d H%d L%d D%d causal=%d  fwd %.3f ms %.0f TF | bwd %.3f ms %.0f TF | torch sdpa fwd %.3f ms %.0f TF"
              " bwd %.3f ms %.0f TF" % (B, H, L, D, causal, tf, fl / tf / 1e9, tb, 2.5 * fl / tb / 1e9, tt,
                                       fl / tt / 1e9, ttb, 2.5 * fl / ttb / 1e9), flush=True)


if __name__ == "__main__":
    main()
