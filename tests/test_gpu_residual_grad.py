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
    monkeypatch.setattr(sa, "_RESID_GRAD_FUSE", True)   # opt-in path (self_attention._RESID_GRAD_FUSE)
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


def test_stacked_blocks_with_layernorm_grad_add(gpu, monkeypatch):
    """Default path (self_attention._LN_GRAD_ADD): each residual dropout_add parks its x-gradient in the
    LayerNorm that produced x (the previous block's output LayerNorm, or the block's first one),
    whose backward kernel sums it with the incoming gradient. Two stacked blocks, so the
    holder handed from one block to the next is exercised; compared with autograd's sums."""
    sa = importlib.import_module("zoo.pipeline.api.keras.layers.self_attention")
    monkeypatch.setattr(importlib.import_module("zoo.ops.nn"), "_DROP_FUSE_MIN", 1)
    monkeypatch.setattr(sa, "_RESID_GRAD_FUSE", False)
    monkeypatch.setattr(sa, "_LN_GRAD_ADD", True)
    torch.manual_seed(0)
    blk = torch.nn.Sequential(sa._Block(256, 4, 1024, 0.1, 0.1, 0.02),
                              sa._Block(256, 4, 1024, 0.1, 0.1, 0.02)).to(gpu).train()
    x = torch.randn(8, 128, 256, device=gpu).to(torch.bfloat16)
    parked = []
    nnm = importlib.import_module("zoo.ops.nn")
    # the residual LayerNorms run as the fused dropout-add LayerNorm (self_attention._DROP_LN_FUSE) or as
    # plain LayerNorms: count a parked gradient in either backward
    for fn in (nnm._LayerNormFn, nnm._DropAddLNFn):
        def spy(ctx, dy, orig=fn.backward):
            if ctx.grad_in is not None and ctx.grad_in.grad is not None:
                parked.append(1)
            return orig(ctx, dy)
        monkeypatch.setattr(fn, "backward", staticmethod(spy))
    gx0, g0 = _grads(blk, x, False, monkeypatch)
    assert not parked
    gx1, g1 = _grads(blk, x, True, monkeypatch)
    assert len(parked) == 3, parked      # block 0 LN1, block 1 LN1, block 0 LN2 (-> block 1's x)
    rel = ((gx1 - gx0).norm() / gx0.norm()).item()
    assert rel < 2e-2, rel
    for k in g0:
        r = ((g1[k] - g0[k]).norm() / g0[k].norm().clamp_min(1e-12)).item()
        assert r < 3e-2, (k, r)
