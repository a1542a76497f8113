"""Run one fused-attention config a few times (for rocprofv3 counter runs).
python tools/attn_one.py B H L D causal [fwd|bwd|both]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from zoo.ops._native import native  # noqa: E402


def main():
    B, H, L, D, causal = (int(a) for a in sys.argv[1:6])
    which = sys.argv[6] if len(sys.argv) > 6 else "both"
    C = native()
    q, k, v = (torch.randn(B, H, L, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    o, lse = C.attn_fwd(q, k, v, None, bool(causal))
    do = torch.randn_like(o)
    for _ in range(3):
        if which in ("fwd", "both"):
            C.attn_fwd(q, k, v, None, bool(causal))
        if which in ("bwd", "both"):
            C.attn_bwd(do, q, k, v, None, o, lse, bool(causal))
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
