"""Fused attention (csrc/kernels/attention.hip) against a plain fp32 PyTorch
reference of softmax(Q K^T / sqrt(D) + mask) V (TransformerLayer.scala:163-181)."""
import math

import pytest
import torch

from zoo.ops.attention import _reference, attention


def _ref32(q, k, v, mask, causal):
    m = None if mask is None else mask[:, None, None, :]
    return _reference(q.float(), k.float(), v.float(), m, causal, 0.0, False)


def test_attention_cpu_reference_matches_manual_softmax():
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 3, 5, 8) for _ in range(3))
    mask = torch.zeros(2, 5)
    mask[1, 3:] = -10000.0
    out = attention(q, k, v, mask=mask, causal=True)
    w = q @ k.transpose(-1, -2) / math.sqrt(8) + mask[:, None, None, :]
    w = w.masked_fill(torch.ones(5, 5, dtype=torch.bool).triu(1), float("-inf"))
    ref = torch.softmax(w, -1) @ v
    assert torch.allclose(out, ref, atol=1e-5)


CASES = [
    # B, H, L, S, D, causal, masked
    (2, 3, 128, 128, 64, False, False),
    (2, 2, 192, 192, 128, True, False),
    (1, 4, 100, 130, 64, False, True),
    (2, 2, 256, 256, 64, True, True),
    (1, 2, 96, 160, 128, False, True),
    (1, 1, 64, 200, 128, True, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,L,S,D,causal,masked", CASES)
def test_fused_attention_matches_fp32(B, H, L, S, D, causal, masked):
    import importlib
    A = importlib.import_module("zoo.ops.attention")
    from zoo.ops._native import native
    assert hasattr(native(), "attn_fwd"), "fused attention kernel not built"
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    q = torch.randn(B, H, L, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, H, S, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, H, S, D, device=dev).to(torch.bfloat16)
    mask = None
    if masked:
        mask = torch.zeros(B, S, device=dev)
        mask[:, S - S // 3:] = -10000.0
    assert A._native_ok(q, k, v, mask, 0.0, False)
    qr, kr, vr = (t.float().detach().requires_grad_(True) for t in (q, k, v))
    ref = _ref32(qr, kr, vr, mask, causal)
    qn, kn, vn = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    out = attention(qn, kn, vn, mask=mask, causal=causal)
    assert out.dtype == torch.bfloat16
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2, err
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.to(torch.bfloat16))
    for name, a, b in (("dq", qn.grad, qr.grad), ("dk", kn.grad, kr.grad), ("dv", vn.grad, vr.grad)):
        rel = (a.float() - b).norm().item() / max(b.norm().item(), 1e-6)
        assert rel < 2e-2, (name, rel)


@pytest.mark.gpu
def test_fused_attention_lse_and_fully_masked_rows():
    from zoo.ops._native import native
    dev = torch.device("cuda:0")
    torch.manual_seed(2)
    q, k, v = (torch.randn(1, 2, 64, 64, device=dev).to(torch.bfloat16) for _ in range(3))
    o, lse = native().attn_fwd(q, k, v, None, False)
    ref = torch.logsumexp((q.float() @ k.float().transpose(-1, -2)) / 8.0, -1)
    assert (lse - ref).abs().max().item() < 1e-2
    # causal with L > S: the first L-S query rows see no key -> zero output
    q2 = torch.randn(1, 1, 128, 64, device=dev).to(torch.bfloat16)
    o2, _ = native().attn_fwd(q2, k[:, :1], v[:, :1], None, True)
    assert o2[:, :, :64].abs().max().item() == 0.0
    assert torch.isfinite(o2.float()).all()


@pytest.mark.gpu
@pytest.mark.parametrize("hd,causal", [(64, False), (64, True), (128, False)])
def test_attention_packed_strided_matches_reference(hd, causal):
    """Fused forward reading q/k/v through strides of one packed [B, L, 3*H*hd]
    projection and writing [B, L, H*hd] (inference path, no head copies)."""
    from zoo.ops.attention import _reference, attention_packed
    torch.manual_seed(0)
    B, L, H = 2, 200, 4
    dev = torch.device("cuda")
    qkv = (torch.randn(B, L, 3 * H * hd, device=dev) * 0.5).bfloat16()
    mask = torch.zeros(B, L, device=dev)
    mask[1, 150:] = -10000.0
    with torch.no_grad():
        out = attention_packed(qkv, H, mask=mask, causal=causal)
    assert out is not None and out.shape == (B, L, H * hd)
    v5 = qkv.float().view(B, L, 3, H, hd).permute(2, 0, 3, 1, 4)
    ref = _reference(v5[0], v5[1], v5[2], mask[:, None, None, :], causal, 0.0, False)
    ref = ref.transpose(1, 2).reshape(B, L, H * hd)
    err = (out.float() - ref).abs().max() / ref.abs().max()
    assert err < 2e-2, err


def _keep_ref(BH, L, S, p, seed):
    """numpy model of the kernel's dropout hash (attention.hip attn_keep): keep-factor [BH, L, S]."""
    import numpy as np
    M = np.uint64(0xFFFFFFFF)

    def fmix(h):
        h = h ^ (h >> np.uint64(16))
        h = (h * np.uint64(0x85EBCA6B)) & M
        h = h ^ (h >> np.uint64(13))
        h = (h * np.uint64(0xC2B2AE35)) & M
        return h ^ (h >> np.uint64(16))

    s0, s1 = np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32)
    bh = np.arange(BH, dtype=np.uint64)[:, None, None]
    q = np.arange(L, dtype=np.uint64)[None, :, None]
    key = np.arange(S, dtype=np.uint64)[None, None, :]
    a = fmix(((bh * np.uint64(0x9E3779B1)) & M) ^ s1)
    h = fmix(((((q * np.uint64(0x85EBCA77)) & M) + key) & M) ^ s0 ^ a)
    thresh = np.uint64(int(p * 4294967296.0))
    return torch.from_numpy((h >= thresh).astype(np.float32) / (1.0 - p))


@pytest.mark.gpu
@pytest.mark.parametrize("D,causal,masked,p", [(64, False, True, 0.1), (64, True, False, 0.5), (128, False, True, 0.1)])
def test_fused_attention_dropout_matches_masked_reference(D, causal, masked, p):
    """In-kernel attention-probability dropout: forward and both backward passes regenerate
    the same counter-hash mask; checked against fp32 autograd through softmax * keep @ V."""
    from zoo.ops._native import native
    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    B, H, L, S = 2, 2, 160, 192
    seed = 0x1234_5678_9ABC
    q = torch.randn(B, H, L, D, device=dev).bfloat16()
    k = torch.randn(B, H, S, D, device=dev).bfloat16()
    v = torch.randn(B, H, S, D, device=dev).bfloat16()
    mask = None
    if masked:
        mask = torch.zeros(B, S, device=dev)
        mask[1, S - 50:] = -10000.0
    keep = _keep_ref(B * H, L, S, p, seed).view(B, H, L, S).to(dev)
    assert abs(float((keep > 0).float().mean()) - (1 - p)) < 0.01
    o, lse = native().attn_fwd(q, k, v, mask, causal, p, seed)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    w = qr @ kr.transpose(-1, -2) / math.sqrt(D)
    if causal:
        w = w.masked_fill(~torch.ones(L, S, dtype=torch.bool, device=dev).tril(S - L), float("-inf"))
    if mask is not None:
        w = w + mask[:, None, None, :]
    ref = (torch.softmax(w, -1) * keep) @ vr
    err = (o.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err
    g = torch.randn_like(ref)
    ref.backward(g)
    dq, dk, dv = native().attn_bwd(g.bfloat16(), q, k, v, mask, o, lse, causal, p, seed)
    for name, a, b in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        rel = (a.float() - b).norm().item() / max(b.norm().item(), 1e-6)
        assert rel < 2e-2, (name, rel)
    # a different seed gives a different output
    o2, _ = native().attn_fwd(q, k, v, mask, causal, p, seed + 1)
    assert (o2.float() - o.float()).abs().max().item() > 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("hd,p", [(64, 0.0), (64, 0.1), (128, 0.1)])
def test_attention_packed_training_grads(hd, p, monkeypatch):
    """Packed training path: strided forward + strided backward writing the packed
    [B, L, 3*H*hd] gradient, vs fp32 autograd of the per-head reference (same dropout mask)."""
    import importlib
    A = importlib.import_module("zoo.ops.attention")   # (zoo.ops.attention the attribute is the function)
    seed = 987654321
    monkeypatch.setattr(A, "_seed", lambda: seed)
    torch.manual_seed(4)
    B, L, H = 2, 136, 4
    dev = torch.device("cuda")
    qkv = (torch.randn(B, L, 3 * H * hd, device=dev) * 0.5).bfloat16().requires_grad_(True)
    mask = torch.zeros(B, L, device=dev)
    mask[0, 100:] = -10000.0
    out = A.attention_packed(qkv, H, mask=mask, causal=False, dropout_p=p, training=True)
    assert out is not None and out.shape == (B, L, H * hd)
    ref_in = qkv.detach().float().requires_grad_(True)
    v5 = ref_in.view(B, L, 3, H, hd).permute(2, 0, 3, 1, 4)
    w = v5[0] @ v5[1].transpose(-1, -2) / math.sqrt(hd) + mask[:, None, None, :]
    pr = torch.softmax(w, -1)
    if p > 0:
        pr = pr * _keep_ref(B * H, L, L, p, seed).view(B, H, L, L).to(dev)
    ref = (pr @ v5[2]).transpose(1, 2).reshape(B, L, H * hd)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.bfloat16())
    rel = (qkv.grad.float() - ref_in.grad).norm().item() / ref_in.grad.norm().item()
    assert rel < 2e-2, rel
