"""The ResNet stem in space-to-depth form on the persistent 1x1 kernel with a gathered operand
(pw.hip EPI 3: 4x4 stride-1 conv, 16 -> 64 channels, BN statistics in the epilogue) against the
fp32 PyTorch conv of the same weights: output and the per-channel (sum, sum of squares)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,H", [(2, 19), (3, 115), (1, 40)])
def test_stem_gather_conv_matches_fp32(gpu, N, H):
    from zoo.ops import _kern
    from zoo.ops.bn import stat_len
    torch.manual_seed(0)
    x = torch.randn(N, H, H, 16, device=gpu).to(torch.bfloat16)
    w = (torch.randn(64, 256, device=gpu) / 16).to(torch.bfloat16)
    stats = torch.zeros(stat_len(64), device=gpu)
    y = _kern.conv_fwd(x, w, 4, 4, stats=stats)
    P = H - 3
    assert y.shape == (N, P, P, 64)
    w4 = w.float().reshape(64, 4, 4, 16).permute(0, 3, 1, 2)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w4).permute(0, 2, 3, 1)
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    assert rel < 5e-3, rel
    yb = y.float().reshape(-1, 64)
    s1, s2 = yb.sum(0), (yb * yb).sum(0)
    torch.testing.assert_close(stats[:64], s1, rtol=1e-3, atol=1e-2 * (N * P * P) ** 0.5)
    torch.testing.assert_close(stats[64:128], s2, rtol=1e-3, atol=1e-2 * (N * P * P) ** 0.5)
