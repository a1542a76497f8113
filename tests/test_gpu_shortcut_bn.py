"""Projection-shortcut BatchNorm fused into the block's last BN apply (ShortcutBN,
bn_fwd_apply resid_bn): outputs, input / parameter gradients and the shortcut's running
statistics must match the unfused block (separate shortcut conv+BN unit) up to bf16
rounding of the skipped intermediate."""
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(block, x, fuse, monkeypatch):
    rn = importlib.import_module("zoo.models.image.resnet")
    monkeypatch.setattr(rn, "FUSE_SHORTCUT_BN", fuse)
    block.zero_grad(set_to_none=True)
    rm0, rv0 = block.down.running_mean.clone(), block.down.running_var.clone()
    xi = x.detach().clone().requires_grad_(True)
    out, _ = block(xi)
    gen = torch.Generator(device=out.device).manual_seed(7)
    w = torch.randn(out.shape, device=out.device, generator=gen)
    (out.float() * w).sum().backward()
    stats = (block.down.running_mean.clone(), block.down.running_var.clone())
    block.down.running_mean.copy_(rm0)
    block.down.running_var.copy_(rv0)
    grads = {k: p.grad.float().clone() for k, p in block.named_parameters() if p.grad is not None}
    return out.float(), xi.grad.float(), grads, stats


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _ref(block, x):
    """fp32 CPU reference of the same block (conv2d_ref / bn_ref path)"""
    import copy
    ref = copy.deepcopy(block).cpu().float().train()
    xi = x.detach().float().cpu().requires_grad_(True)
    out = ref(xi)
    out = out[0] if isinstance(out, tuple) else out
    gen = torch.Generator(device=x.device).manual_seed(7)
    w = torch.randn(out.shape, device=x.device, generator=gen).cpu()
    (out * w).sum().backward()
    grads = {k: p.grad.float().clone() for k, p in ref.named_parameters() if p.grad is not None}
    return out, xi.grad, grads


@pytest.mark.parametrize("kind,cin,width,stride", [("bottleneck", 64, 32, 2), ("bottleneck", 64, 64, 1),
                                                    ("basic", 32, 64, 2)])
def test_fused_shortcut_bn_matches_unfused(gpu, monkeypatch, kind, cin, width, stride):
    """the fused path is as close to the fp32 reference as the unfused bf16 path"""
    rn = importlib.import_module("zoo.models.image.resnet")
    torch.manual_seed(0)
    blk = (rn.Bottleneck(cin, width, stride) if kind == "bottleneck" else rn.BasicBlock(cin, width, stride))
    blk = blk.to(gpu).train()
    with torch.no_grad():
        blk.down.gamma.uniform_(0.5, 1.5)
        blk.down.beta.uniform_(-0.5, 0.5)
    x = torch.randn(8, 28, 28, cin, device=gpu).to(torch.bfloat16)
    orf, gxr, gr = _ref(blk, x)
    o0, gx0, g0, s0 = _run(blk, x, False, monkeypatch)
    o1, gx1, g1, s1 = _run(blk, x, True, monkeypatch)

    def close(a1, a0, r, what):
        e1, e0 = _rel(a1.cpu(), r), _rel(a0.cpu(), r)
        assert e1 <= 1.25 * e0 + 5e-3, (what, e1, e0)

    close(o1, o0, orf.float(), "out")
    close(gx1, gx0, gxr.float(), "dx")
    assert set(g0) == set(g1)
    for k in g0:
        close(g1[k], g0[k], gr[k].float(), k)
    assert torch.allclose(s1[0], s0[0], rtol=1e-4, atol=1e-5)
    assert torch.allclose(s1[1], s0[1], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mask_form", ["bits", "z"])
def test_consumer_epilogue_second_bn_sums(gpu, mask_form):
    """BNProducer.y2: the consumer conv's BN-backward epilogue also sums out * y2 per channel
    (pw.hip EPI 2 for the 1-bit mask form; the bf16-z form runs on another kernel and gets the
    sums from one reduction pass) -- against fp32 torch, main BN sums included."""
    from zoo.ops import _kern
    from zoo.ops.bn import stat_len
    torch.manual_seed(3)
    N, H, W, Ci, Co = 2, 14, 14, 64, 256
    x = (torch.randn(N, H, W, Ci, device=gpu) * 0.5).bfloat16()
    w = (torch.randn(Co, Ci, device=gpu) * 0.1).bfloat16()
    y = torch.randn(N, H, W, Co, device=gpu).bfloat16()
    y2 = torch.randn(N, H, W, Co, device=gpu).bfloat16()
    pre = torch.randn(N, H, W, Co, device=gpu)
    keep = pre > 0
    mean = torch.randn(Co, device=gpu) * 0.1
    inv = torch.rand(Co, device=gpu) + 0.5
    sums = torch.zeros(stat_len(Co), device=gpu)
    sums2 = torch.zeros(Co, device=gpu)
    if mask_form == "bits":
        bits = (keep.view(-1, 8).int() << torch.arange(8, device=gpu)).sum(1).to(torch.uint8)
        zarg = bits
    else:
        zarg = torch.where(keep, pre.abs() + 0.1, torch.zeros_like(pre)).bfloat16()
    out = _kern.conv_fwd(x, w, 1, 1, bstats=(zarg, y, mean, inv, sums, None, None, y2, sums2))
    o = (x.float().reshape(-1, Ci) @ w.float().t()).reshape(N, H, W, Co) * keep
    ob = o.bfloat16().float()
    assert _rel(out.float().cpu(), o.cpu()) < 1e-2
    ref2 = (ob * y2.float()).reshape(-1, Co).sum(0)
    ref_s1 = ob.reshape(-1, Co).sum(0)
    ref_s2 = (ob * (y.float() - mean) * inv).reshape(-1, Co).sum(0)
    assert _rel(sums2.cpu(), ref2.cpu()) < 2e-3
    assert _rel(sums[:Co].cpu(), ref_s1.cpu()) < 2e-3 and _rel(sums[Co:2 * Co].cpu(), ref_s2.cpu()) < 2e-3
