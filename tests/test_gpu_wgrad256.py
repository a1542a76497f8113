"""256x256-tile weight-gradient kernel (csrc/kernels/wgrad256.hip, ``zoo._C.linear_wgrad``):
dW (fp32) += dY^T X against a float64 reference, over shapes that exercise the split
fold, single-split direct accumulation, ragged N / K / M edges and strided operands."""
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [
    (16384, 768, 768),      # many splits, fold
    (4096, 2304, 768),
    (1000, 264, 520),       # ragged tiles and a partial last m-step
    (64, 256, 256),         # single split: direct accumulate
    (200, 8, 16),           # tiny
    (70000, 64, 256),       # long reduction (ResNet 1x1 shape class)
    (200704, 512, 128),     # ResNet stage-2 1x1: atomic split-K (half-live tiles)
])
@pytest.mark.parametrize("det", [False, True])   # True: partials + ordered fold; False: atomics where small
def test_linear_wgrad_matches_fp64(M, N, K, det):
    from zoo.ops._native import native
    dev = torch.device("cuda")
    torch.manual_seed(M + N + K)
    dy = (torch.randn(M, N, device=dev) * 0.1).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    init = torch.randn(N, K, device=dev)
    dw = init.clone()
    native().set_deterministic(det)
    try:
        native().linear_wgrad(dy, x, dw)
    finally:
        native().set_deterministic(False)
    ref = init.double() + dy.double().t() @ x.double()
    err = ((dw.double() - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err


@pytest.mark.gpu
def test_linear_wgrad_strided_operands_and_padded_dw():
    from zoo.ops._native import native
    dev = torch.device("cuda")
    torch.manual_seed(7)
    M, N, K = 3000, 384, 136
    big_dy = (torch.randn(M, N + 64, device=dev) * 0.1).bfloat16()
    big_x = torch.randn(M, K + 40, device=dev).bfloat16()
    dy, x = big_dy[:, 32:32 + N], big_x[:, :K]
    dw_full = torch.zeros(N, K + 24, device=dev)
    native().linear_wgrad(dy, x, dw_full)
    ref = dy.double().t() @ x.double()
    assert ((dw_full[:, :K].double() - ref).norm() / ref.norm()).item() < 1e-5
    assert dw_full[:, K:].abs().max().item() == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("act", [None, "relu", "gelu"])
@pytest.mark.parametrize("flat", [False, True])
def test_blas_linear_backward_matches_fp32(act, flat):
    """Transformer-size linear layer (hipBLASLt forward, native backward pieces: fused
    activation-backward + bias column sums, wgrad256 weight gradient) against fp32 autograd,
    with and without an engine-owned flat fp32 gradient buffer."""
    from zoo import ops
    dev = torch.device("cuda")
    torch.manual_seed(11)
    M, Cin, K = 2048, 512, 768
    x = (torch.randn(M, Cin, device=dev)).bfloat16().requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(K, Cin, device=dev) * 0.05)
    b = torch.nn.Parameter(torch.randn(K, device=dev) * 0.1)
    if flat:
        w._zoo_grad = torch.zeros(K * Cin, device=dev)
        b._zoo_grad = torch.zeros(K, device=dev)
    y = ops.linear(x, w, b, act=act)
    g = torch.randn(M, K, device=dev).bfloat16()
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr.bfloat16().float(), br)
    if act == "relu":
        yr = torch.relu(yr)
    elif act == "gelu":
        yr = torch.nn.functional.gelu(yr)
    yr.backward(g.float())
    assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2
    gw = w._zoo_grad.view(K, Cin) if flat else w.grad
    gb = b._zoo_grad if flat else b.grad
    for name, a, r in (("dx", x.grad, xr.grad), ("dw", gw, wr.grad), ("db", gb, br.grad)):
        rel = ((a.float() - r).norm() / r.norm()).item()
        assert rel < 2e-2, (name, rel)
