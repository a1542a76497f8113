#!/usr/bin/env python3
"""Isolated conv->BN->ReLU unit (native_nets.CBR) on the GPU vs its CPU fp32 reference with the
SAME input and upstream gradient: dgamma / dbeta / dweight / dx relative errors, for the unit's
standalone BN-backward path (no fused consumer) -- the layer_parity.py suspects."""
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def rel(a, b):
    a, b = a.detach().float().cpu().flatten(), b.detach().float().cpu().flatten()
    return round(float((a - b).norm() / b.norm().clamp_min(1e-20)), 5)


def main():
    from zoo.models.image.native_nets import CBR
    dev = torch.device("cuda")
    for (cin, cout, k, s, p, hw, n) in [(32, 64, 1, 1, 0, 112, 2), (16, 32, 3, 2, 1, 224, 2), (64, 128, 1, 1, 0, 56, 8),
                                        (256, 256, 3, 1, 1, 14, 4)]:
        torch.manual_seed(0)
        u = CBR(cin, cout, k, s, p)
        c = copy.deepcopy(u).train()
        g = copy.deepcopy(u).to(dev).train()
        x = torch.randn(n, hw, hw, cin).bfloat16().float()
        xc = x.clone().requires_grad_(True)
        yc = c(xc)
        dy = torch.randn_like(yc).bfloat16().float()
        yc.backward(dy)
        xg = x.to(dev).bfloat16().requires_grad_(True)
        yg = g(xg)
        yg.backward(dy.to(dev).to(yg.dtype))
        torch.cuda.synchronize()
        print(json.dumps({"unit": [cin, cout, k, s, p, hw, n], "fwd": rel(yg, yc), "dx": rel(xg.grad, xc.grad),
                          "dweight": rel(g.weight.grad, c.weight.grad), "dgamma": rel(g.gamma.grad, c.gamma.grad),
                          "dbeta": rel(g.beta.grad, c.beta.grad)}), flush=True)


if __name__ == "__main__":
    main()
