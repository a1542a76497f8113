"""GELU backward in the consuming linear's data-gradient epilogue (zoo.ops.nn.GeluLink,
csrc/kernels/igemm*.hip EPI 2 with BwdStats.zgelu): the FFN pair fc2(gelu(fc1(x))) gives the
fp32 reference gradients, the separate activation-backward pass is gone from the trace, and a
Transformer block matches the unfused path."""
import importlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ffn(x, w1, b1, w2, b2, link):
    from zoo import ops
    m = ops.linear(x, w1, b1, act="gelu", gelu_link=link)
    return ops.linear(m, w2, b2, gelu_src=link)


@pytest.mark.parametrize("M,H,I", [(2048, 256, 1024), (4096, 768, 3072)])
def test_ffn_pair_matches_fp32(gpu, M, H, I, monkeypatch):
    from torch.profiler import ProfilerActivity, profile
    from zoo.ops import conv
    from zoo.ops.nn import GeluLink
    monkeypatch.setattr(conv, "_GELU_DGRAD", True)
    torch.manual_seed(0)
    x = torch.randn(M, H, device=gpu).to(torch.bfloat16)
    w1 = (torch.randn(I, H, device=gpu) * 0.03).requires_grad_(True)
    b1 = (torch.randn(I, device=gpu) * 0.1).requires_grad_(True)
    w2 = (torch.randn(H, I, device=gpu) * 0.03).requires_grad_(True)
    b2 = (torch.randn(H, device=gpu) * 0.1).requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    g = torch.randn(M, H, device=gpu)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        y = _ffn(xg, w1, b1, w2, b2, GeluLink())
        (y.float() * g).sum().backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert not [n for n in names if "act_colsum_kernel<2" in n], "separate GELU backward still ran"
    assert not [n for n in names if "Cijk_" in n]
    # fp32 reference from the same bf16 operands
    xr = x.float().requires_grad_(True)
    p = [t.detach().float().requires_grad_(True) for t in (w1, b1, w2, b2)]
    yr = F.linear(F.gelu(F.linear(xr, p[0], p[1])), p[2], p[3])
    (yr * g).sum().backward()
    assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2
    for got, ref, nm in ((xg.grad, xr.grad, "x"), (w1.grad, p[0].grad, "w1"), (b1.grad, p[1].grad, "b1"),
                         (w2.grad, p[2].grad, "w2"), (b2.grad, p[3].grad, "b2")):
        r = ((got.float() - ref).norm() / ref.norm()).item()
        assert r < 2e-2, (nm, r)


def test_block_matches_unfused(gpu, monkeypatch):
    sa = importlib.import_module("zoo.pipeline.api.keras.layers.self_attention")
    conv = importlib.import_module("zoo.ops.conv")
    nn_mod = importlib.import_module("zoo.ops.nn")
    torch.manual_seed(0)
    blk = sa._Block(256, 4, 1024, 0.0, 0.0, 0.02).to(gpu).train()
    x = torch.randn(8, 128, 256, device=gpu).to(torch.bfloat16)
    out = {}
    for fuse in (False, True):
        monkeypatch.setattr(conv, "_GELU_DGRAD", fuse)
        nn_mod._DROP_RNG.clear()
        blk.zero_grad(set_to_none=True)
        xi = x.detach().clone().requires_grad_(True)
        y = blk(xi)
        w = torch.linspace(-1, 1, y.numel(), device=gpu).reshape(y.shape)
        (y.float() * w).sum().backward()
        out[fuse] = (y.float(), xi.grad.float(), {k: p.grad.float().clone() for k, p in blk.named_parameters()})
    (y0, gx0, g0), (y1, gx1, g1) = out[False], out[True]
    assert torch.equal(y0, y1)
    assert ((gx1 - gx0).norm() / gx0.norm()).item() < 2e-2
    for k in g0:
        r = ((g1[k] - g0[k]).norm() / g0[k].norm().clamp_min(1e-12)).item()
        assert r < 3e-2, (k, r)


@pytest.mark.parametrize("M,K,N", [(16384, 768, 3072), (4096, 768, 3072), (512, 96, 136)])
def test_gelu_linear_stores_pre_activation_from_the_epilogue(gpu, M, K, N):
    """conv_fwd(act=GELU, act_pre=...): the output gelu(v) and the bf16 pre-activation v from one
    GEMM (igemm2.hip EPI 3 dual store) -- no separate GELU pass in the trace on the large-tile
    shapes; a shape that kernel does not take (512 x 96 x 136) runs GEMM + GELU pass instead.
    Both against fp32 PyTorch."""
    from torch.profiler import ProfilerActivity, profile
    from zoo.ops import _kern
    torch.manual_seed(2)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = (torch.randn(N, K, device=gpu) * 0.05).bfloat16()
    b = torch.randn(N, device=gpu) * 0.1
    pre = torch.empty(M, 1, 1, N, dtype=torch.bfloat16, device=gpu)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        y = _kern.conv_fwd(x.view(M, 1, 1, K), w, 1, 1, bias=b, act=2, act_pre=pre)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    vref = x.float() @ w.float().t() + b
    assert (pre.view(M, N).float() - vref).abs().max().item() <= 1e-2 * vref.abs().max().item()
    yref = F.gelu(pre.view(M, N).float())                 # GELU of the stored (rounded) value
    assert (y.view(M, N).float() - yref).abs().max().item() <= 1e-2 * yref.abs().max().item()
    if M >= 4096:
        assert any("igemm2_kernel" in n for n in names), names
        assert not [n for n in names if "act_kernel" in n], names
