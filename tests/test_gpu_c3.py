"""Numerics of the persistent streaming 3x3 conv (csrc/kernels/c3.hip: stride 1, pad 1,
64 -> 64 channels, the ResNet stage-1 3x3) against plain PyTorch fp32 references:

  * forward + BN statistics, whole images per workgroup and images split into runs of bands
    (small batches), a partial last band (H not a multiple of the 4-row band), more work items
    than workgroups, and the deterministic partial-row statistics mode;
  * data gradient with the fused BN-backward epilogue in every producer-mask mode (ReLU
    recomputed from y and the producer affine, 1-bit mask, bf16 z) and a residual gradient.
Each case is also run with the kernel switched off (c3_set(0): igemm2 / igemm) and compared.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture
def C3(gpu):
    from zoo.ops import native
    C = native()
    yield C
    C.c3_set(-1)
    C.set_deterministic(False)


def _conv(C, x, w2, stats):
    return C.conv_fwd(x, w2, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, None, None, stats, 0, False, True, 0, 0, None, [],
                      None, None, None, None, None)


@pytest.mark.parametrize("N,H", [(2, 56), (1, 56), (40, 56), (3, 18), (300, 56)])
def test_c3_fwd_stats(C3, gpu, N, H):
    torch.manual_seed(N + H)
    x = torch.randn(N, H, 56, 64, device=gpu).bfloat16()
    w4 = (torch.randn(64, 3, 3, 64, device=gpu) / math.sqrt(576)).bfloat16()
    w2 = w4.reshape(64, -1).contiguous()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w4.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert C3.c3_grid_for(N, H, 56) > 0
    C3.c3_set(1)
    stats = torch.zeros(2 * 64, device=gpu)
    y = _conv(C3, x, w2, stats)
    assert rel(y, ref) < 1e-2
    yf = y.float()
    assert rel(stats, torch.cat([yf.sum((0, 1, 2)), (yf * yf).sum((0, 1, 2))])) < 1e-3
    C3.c3_set(0)
    y0 = _conv(C3, x, w2, None)
    assert rel(y, y0) < 1e-2


def test_c3_deterministic_partial_stats(C3, gpu):
    torch.manual_seed(3)
    x = torch.randn(8, 56, 56, 64, device=gpu).bfloat16()
    w2 = (torch.randn(64, 576, device=gpu) / 24.0).bfloat16()
    C3.c3_set(1)
    C3.set_deterministic(True)
    outs = []
    for _ in range(2):
        stats = torch.zeros(2 * 64, device=gpu)
        y = _conv(C3, x, w2, stats)
        outs.append((y, stats))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    yf = outs[0][0].float()
    assert rel(outs[0][1], torch.cat([yf.sum((0, 1, 2)), (yf * yf).sum((0, 1, 2))])) < 1e-3


@pytest.mark.parametrize("zmode", ["affine", "bits", "z", "none"])
@pytest.mark.parametrize("with_resid", [False, True])
def test_c3_dgrad_fused_bn_backward(C3, gpu, zmode, with_resid):
    from zoo.ops import _kern
    N, H, W = 4, 56, 56
    torch.manual_seed(7)
    y_pre = torch.randn(N, H, W, 64, device=gpu).bfloat16()
    mean = y_pre.float().mean((0, 1, 2))
    inv = torch.rsqrt(y_pre.float().var((0, 1, 2), unbiased=False) + 1e-5)
    gamma = torch.rand(64, device=gpu) + 0.5
    beta = torch.randn(64, device=gpu) * 0.1
    pre = (y_pre.float() - mean) * inv * gamma + beta
    z = torch.relu(pre).bfloat16()
    w4 = (torch.randn(64, 3, 3, 64, device=gpu) / math.sqrt(576)).bfloat16()
    w2 = w4.reshape(64, -1).contiguous()
    dy = torch.randn(N, H, W, 64, device=gpu).bfloat16()
    resid = torch.randn(N, H, W, 64, device=gpu).bfloat16() if with_resid else None
    zr = z.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(zr, w4.float().permute(0, 3, 1, 2), padding=1).backward(dy.float().permute(0, 3, 1, 2))
    dz = zr.grad.permute(0, 2, 3, 1) + (resid.float() if resid is not None else 0.0)
    sums = torch.zeros(2 * 64, device=gpu)
    if zmode == "none":
        bst, ref = None, dz
    else:
        keep = (pre > 0) if zmode == "affine" else (z.float() > 0)
        ref = dz * keep
        if zmode == "z":
            bst = (z, y_pre, mean.contiguous(), inv.contiguous(), sums)
        elif zmode == "affine":
            bst = (None, y_pre, mean.contiguous(), inv.contiguous(), sums, gamma, beta)
        else:
            bits = (z.view(-1, 8) > 0).to(torch.uint8)
            packed = (bits << torch.arange(8, device=gpu, dtype=torch.uint8)).sum(1).to(torch.uint8)
            bst = (packed.contiguous(), y_pre, mean.contiguous(), inv.contiguous(), sums)
    C3.c3_set(1)
    out = _kern.conv_dgrad(dy, w2, 64, 3, 3, 64, H, W, (1, 1), (1, 1), resid=resid, bstats=bst)
    assert rel(out, ref) < 1e-2
    if bst is not None:
        q = out.float()
        xhat = (y_pre.float() - mean) * inv
        assert rel(sums, torch.cat([q.sum((0, 1, 2)), (q * xhat).sum((0, 1, 2))])) < 2e-3
    C3.c3_set(0)
    out0 = _kern.conv_dgrad(dy, w2, 64, 3, 3, 64, H, W, (1, 1), (1, 1), resid=resid,
                            bstats=None if bst is None else tuple(
                                torch.zeros_like(t) if (t is sums) else t for t in bst))
    assert rel(out, out0) < 1e-2
