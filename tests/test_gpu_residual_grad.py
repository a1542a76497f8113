"""Transformer residual-gradient handoff (zoo.ops.nn.GradAdd): the residual add's
x-gradient folded into the consuming linear's data-gradient GEMM must give the same
gradients as autograd's separate sum (bf16 GEMM rounding only), with dropout on."""
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(block, x, use_handoff, monkeypatch):
    sa = importlib.import_module("zoo.pipeline.api.keras.layers.self_attention")
    nn_mod = importlib.import_module("zoo.ops.nn")
    if not use_handoff:
        monkeypatch.setattr(sa, "GradAdd", lambda: None)
    else:
        monkeypatch.setattr(sa, "GradAdd", nn_mod.GradAdd)
    nn_mod._DROP_RNG.clear()          # identical dropout masks in both runs (residual and attention)
    importlib.import_module("zoo.ops.pointwise")._RNG.clear()
    block.zero_grad(set_to_none=True)
    xi = x.detach().clone().requires_grad_(True)
    y = block(xi)
    w = torch.linspace(-1, 1, y.numel(), device=y.device).reshape(y.shape).to(y.dtype)
    (y.float() * w.float()).sum().backward()
    return xi.grad.float(), {k: p.grad.float().clone() for k, p in block.named_parameters() if p.grad is not None}


def test_block_grads_with_residual_handoff(gpu, monkeypatch):
    sa = importlib.import_module("zoo.pipeline.api.keras.layers.self_attention")
    monkeypatch.setattr(importlib.import_module("zoo.ops.nn"), "_DROP_FUSE_MIN", 1)
    monkeypatch.setattr(sa, "_RESID_GRAD_FUSE", True)   # opt-in path (ZOO_RESID_GRAD_FUSE=1)
    torch.manual_seed(0)
    blk = sa._Block(256, 4, 1024, 0.1, 0.1, 0.02).to(gpu).train()
    x = torch.randn(8, 128, 256, device=gpu).to(torch.bfloat16)
    gx0, g0 = _grads(blk, x, False, monkeypatch)
    gx1, g1 = _grads(blk, x, True, monkeypatch)
    rel = ((gx1 - gx0).norm() / gx0.norm()).item()
    assert rel < 2e-2, rel
    for k in g0:
        r = ((g1[k] - g0[k]).norm() / g0[k].norm().clamp_min(1e-12)).item()
        assert r < 3e-2, (k, r)
