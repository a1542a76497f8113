"""Streaming 1x1 conv kernel (csrc/kernels/pw.hip) against a plain PyTorch fp32 reference of the
same op: the forward with BatchNorm statistics (EPI 1) and the data gradient with the fused
BN-backward epilogue (EPI 2: recomputed ReLU mask / 1-bit mask + residual-gradient add, sums).
Row counts that are not a multiple of the wave tile exercise the tails."""
import pytest
import torch

pytestmark = pytest.mark.gpu

FWD = [(64, 64), (64, 128), (64, 256), (128, 128), (128, 512), (256, 64), (512, 128), (1024, 256), (2048, 512)]
BWD = [(64, 64), (64, 256), (128, 512), (256, 64), (512, 128), (1024, 256), (256, 512)]


def _native():
    from zoo.ops._native import native
    return native()


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("N,K", FWD)
def test_pw_forward_stats(gpu, N, K):
    from zoo.ops import _kern
    C = _native()
    g = torch.Generator(device="cuda").manual_seed(N + K)
    x = torch.randn(3, 19, 23, K, device="cuda", generator=g).bfloat16()      # M = 1311
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    C.pw_set(1)
    try:
        stats = torch.zeros(C.stat_len(N), device="cuda")
        y = _kern.conv_fwd(x, w, 1, 1, stats=stats)
        torch.cuda.synchronize()
    finally:
        C.pw_set(-1)
    ref = (x.float().reshape(-1, K) @ w.float().t())
    assert _rel(y.reshape(-1, N), ref) < 1e-2
    yq = y.float().reshape(-1, N)
    assert torch.allclose(stats[:N], yq.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(stats[N:2 * N], (yq * yq).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("N,K", BWD)
@pytest.mark.parametrize("mode", ["z1", "z2r"])
def test_pw_dgrad_bn_backward(gpu, N, K, mode):
    """dgrad of a 1x1 conv N->K (output has N channels) with the producer's BN-backward fused."""
    from zoo.ops import _kern
    C = _native()
    g = torch.Generator(device="cuda").manual_seed(7 * N + K)
    shape = (2, 17, 29)                                                        # M = 986
    dy = torch.randn(*shape, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(K, N, device="cuda", generator=g) / N ** 0.5).bfloat16()  # conv weight [Cout=K][Cin=N]
    y = torch.randn(*shape, N, device="cuda", generator=g).bfloat16()
    mean = torch.randn(N, device="cuda", generator=g) * 0.1
    inv = torch.rand(N, device="cuda", generator=g) + 0.5
    gam = torch.rand(N, device="cuda", generator=g) + 0.5
    bet = torch.randn(N, device="cuda", generator=g) * 0.2
    M = dy.numel() // K
    bits = torch.randint(0, 2, (M, N), device="cuda", generator=g, dtype=torch.uint8)
    mask = (bits.reshape(-1, 8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    resid = torch.randn(*shape, N, device="cuda", generator=g).bfloat16() if mode == "z2r" else None
    sums = torch.zeros(C.stat_len(N), device="cuda")
    bst = (None, y, mean, inv, sums, gam, bet) if mode == "z1" else (mask, y, mean, inv, sums)
    C.pw_set(1)
    try:
        dx = _kern.conv_dgrad(dy, w, K, 1, 1, N, shape[1], shape[2], resid=resid, bstats=bst)
        torch.cuda.synchronize()
    finally:
        C.pw_set(-1)
    v = dy.float().reshape(-1, K) @ w.float()
    if resid is not None:
        v = v + resid.float().reshape(-1, N)
    yf = y.float().reshape(-1, N)
    if mode == "z1":
        sc = gam * inv
        keep = (yf * sc + (bet - mean * sc)) > 0
    else:
        keep = bits.bool()
    v = torch.where(keep, v, torch.zeros_like(v))
    assert _rel(dx.reshape(-1, N), v) < 1e-2
    q = dx.float().reshape(-1, N)
    assert torch.allclose(sums[:N], q.sum(0), rtol=1e-3, atol=5e-2)
    assert torch.allclose(sums[N:2 * N], (q * (yf - mean) * inv).sum(0), rtol=1e-3, atol=5e-2)


def test_pw_matches_tiled_kernels(gpu):
    """Same call through pw.hip and through igemm / igemm2 (pw off): identical up to fp32 sum order."""
    from zoo.ops import _kern
    C = _native()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(4, 28, 28, 256, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 256, device="cuda", generator=g) / 16).bfloat16()
    outs = []
    for mode in (1, 0):
        C.pw_set(mode)
        st = torch.zeros(C.stat_len(64), device="cuda")
        outs.append((_kern.conv_fwd(x, w, 1, 1, stats=st), st[:128].clone()))
    C.pw_set(-1)
    torch.cuda.synchronize()
    assert _rel(outs[0][0], outs[1][0]) < 1e-2
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-3, atol=1e-1)
