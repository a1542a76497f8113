"""Fused Transformer residual LayerNorm (ops.nn.dropout_add_layer_norm: one native pass for
LayerNorm(x + dropout(a))) against the two-op path it replaces (dropout_add, then layer_norm)
drawing the same host seed, and against an fp32 PyTorch reference built from the mask that path
applies. Reference: TransformerLayer.scala:129-181 (residual dropout + LayerNorm)."""
import random

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _reseed(seed):
    from zoo.ops import nn as N
    N._DROP_RNG[:] = [random.Random(seed)]


@pytest.mark.parametrize("rows,D", [(16384, 768), (4096, 1024), (8192, 512)])
def test_fused_dropout_add_layernorm_matches_two_op_path(gpu, rows, D):
    from zoo.ops import nn as N
    torch.manual_seed(rows + D)
    p = 0.1
    a0 = torch.randn(rows, D, device=gpu).bfloat16()
    x0 = torch.randn(rows, D, device=gpu).bfloat16()
    g0 = (torch.rand(D, device=gpu) + 0.5)
    b0 = torch.randn(D, device=gpu) * 0.1
    dy = torch.randn(rows, D, device=gpu).bfloat16()
    outs = []
    for fused in (True, False):
        a, x = a0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
        g, b = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        _reseed(11)
        if fused:
            y = N.dropout_add_layer_norm(a, x, p, True, g, b, 1e-5)
            assert y.grad_fn is not None and "DropAddLN" in type(y.grad_fn).__name__
        else:
            y = N.layer_norm(N.dropout_add(a, x, p, True), g, b, 1e-5)
        y.backward(dy)
        outs.append((y.detach(), a.grad, x.grad, g.grad, b.grad))
    (yf, daf, dxf, dgf, dbf), (yu, dau, dxu, dgu, dbu) = outs
    assert torch.equal(yf, yu)
    assert torch.equal(daf, dau) and torch.equal(dxf, dxu)
    assert torch.allclose(dgf, dgu, rtol=1e-4, atol=1e-3) and torch.allclose(dbf, dbu, rtol=1e-4, atol=1e-3)
    # fp32 reference with the same mask (recovered from the two-op path's dropout output)
    _reseed(11)
    from zoo.ops._native import native
    seed = N._drop_rng().getrandbits(62)
    keep = native().dropout_add(torch.ones_like(a0), None, p, seed).float() > 0
    frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01
    s = x0.float() + a0.float() * keep / (1 - p)
    ref = F.layer_norm(s, (D,), g0, b0, 1e-5)
    assert ((yf.float() - ref).abs().max() / ref.abs().max()).item() < 2e-2


def test_bert_block_uses_fused_residual_layernorm(gpu):
    """One BERT block forward/backward with the fused op on and off gives the same outputs and
    parameter gradients under the same dropout seeds."""
    from zoo.pipeline.api.keras.layers import self_attention as SA
    torch.manual_seed(0)
    blk = SA._Block(768, 12, 3072, 0.1, 0.0, 0.02).to(gpu).train()
    x0 = torch.randn(64, 128, 768, device=gpu).bfloat16()   # above the fused-dropout size floor
    res = []
    for fused in (True, False):
        SA._DROP_LN_FUSE = fused
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            _reseed(5)
            y = blk(x)
            (y.float() ** 2).mean().backward()
            res.append((y.detach().float(), x.grad.float(), {k: v.grad.float() for k, v in blk.named_parameters()}))
        finally:
            SA._DROP_LN_FUSE = True
    (y1, dx1, g1), (y2, dx2, g2) = res
    assert (y1 - y2).abs().max().item() < 1e-2
    assert ((dx1 - dx2).norm() / dx2.norm()).item() < 1e-2
    for k in g1:
        assert ((g1[k] - g2[k]).norm() / g2[k].norm().clamp_min(1e-12)).item() < 2e-2, k
