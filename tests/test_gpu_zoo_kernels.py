"""Round-2 kernels for the model zoo and the Keras layers, each against a plain
PyTorch fp32 reference of the same op (forward and backward): depthwise conv,
NHWC average pooling (ceil mode / count_include_pad), ceil-mode max pooling,
row softmax / log-softmax, cross-channel LRN."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("C,H,k,stride,pad", [(32, 14, 3, 1, 1), (96, 15, 3, 2, 1), (144, 8, 3, 1, 0),
                                              (64, 9, 1, 1, 0), (40, 10, 2, 2, 0),
                                              # sliding-window 3x3 wgrad: wide rows, 2-channel-chunk
                                              # groups, 1024 / 960 channels on 7x7, odd sizes
                                              (32, 112, 3, 1, 1), (8, 57, 3, 2, 1), (1024, 7, 3, 1, 1),
                                              (960, 7, 3, 1, 1), (24, 113, 3, 2, 1)])
def test_depthwise_conv_fwd_bwd(gpu, C, H, k, stride, pad):
    from zoo.ops.nn import depthwise_conv2d_nhwc
    N = 3
    x = torch.randn(N, H, H, C, device=gpu).bfloat16()
    w = (torch.randn(k * k, C, device=gpu) * 0.3).requires_grad_(True)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.detach().t().reshape(C, 1, k, k).clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=stride, padding=pad, groups=C)
    xg = x.detach().clone().requires_grad_(True)
    y = depthwise_conv2d_nhwc(xg, w, kernel=(k, k), stride=(stride, stride), pad=(pad, pad))
    assert y.shape == (N, yr.shape[2], yr.shape[3], C)
    assert rel(y, yr.permute(0, 2, 3, 1)) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert rel(xg.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert rel(w.grad, wr.grad.reshape(C, k * k).t()) < 1e-2


def test_depthwise_wgrad_deterministic(gpu):
    from zoo.ops.nn import depthwise_conv2d_nhwc
    x = torch.randn(8, 56, 56, 128, device=gpu).bfloat16()
    dy = torch.randn(8, 56, 56, 128, device=gpu).bfloat16()
    grads = []
    for _ in range(2):
        w = torch.randn(9, 128, device=gpu).requires_grad_(True)
        torch.manual_seed(0)
        with torch.no_grad():
            w.copy_(torch.randn(9, 128, device=gpu))
        depthwise_conv2d_nhwc(x, w, kernel=(3, 3), stride=(1, 1), pad=(1, 1)).backward(dy)
        grads.append(w.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_depthwise_conv_relu_bias(gpu):
    from zoo.ops.nn import depthwise_conv2d_nhwc
    x = torch.randn(2, 7, 7, 24, device=gpu).bfloat16()
    w = torch.randn(9, 24, device=gpu) * 0.3
    b = torch.randn(24, device=gpu)
    y = depthwise_conv2d_nhwc(x, w, b, (3, 3), (1, 1), (1, 1), act="relu")
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.t().reshape(24, 1, 3, 3), b, padding=1, groups=24))
    assert rel(y, ref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("k,s,p,ceil,inc", [(2, 2, 0, False, True), (3, 2, 1, True, True), (3, 1, 1, False, False),
                                            (3, 2, 0, True, False)])
def test_avg_pool_fwd_bwd(gpu, k, s, p, ceil, inc):
    from zoo.ops.pool import avg_pool2d_nhwc
    x = torch.randn(2, 13, 13, 16, device=gpu).bfloat16()
    # reference on the CPU: ROCm torch's ceil-mode avg_pool2d backward disagrees with its own CPU path
    xr = x.float().cpu().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.avg_pool2d(xr, k, s, p, ceil_mode=ceil, count_include_pad=inc)
    xg = x.detach().clone().requires_grad_(True)
    y = avg_pool2d_nhwc(xg, (k, k), (s, s), (p, p), ceil_mode=ceil, count_include_pad=inc)
    assert y.shape == (2, yr.shape[2], yr.shape[3], 16)
    assert rel(y.cpu(), yr.permute(0, 2, 3, 1)) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float().cpu().permute(0, 3, 1, 2))
    assert rel(xg.grad.cpu(), xr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_max_pool_ceil_mode(gpu):
    from zoo.ops.pool import max_pool2d_nhwc
    x = torch.randn(2, 14, 14, 32, device=gpu).bfloat16()
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 0, ceil_mode=True)
    xg = x.detach().clone().requires_grad_(True)
    y = max_pool2d_nhwc(xg, (3, 3), (2, 2), (0, 0), ceil_mode=True)
    assert y.shape == (2, yr.shape[2], yr.shape[3], 32)
    assert rel(y, yr.permute(0, 2, 3, 1)) < 1e-3
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert rel(xg.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("N,H,W,C,k,s,p,ceil", [(2, 112, 112, 64, 3, 2, 1, False),   # ResNet stem
                                                 (3, 17, 13, 128, 2, 2, 0, False),
                                                 (2, 15, 15, 8, 3, 2, 1, True),
                                                 (1, 9, 20, 256, 3, 1, 1, False),
                                                 (2, 11, 11, 48, 3, 2, 1, False)])    # C/8 = 6: grid-stride kernel
def test_max_pool_row_kernels(gpu, N, H, W, C, k, s, p, ceil):
    """Row-per-block max-pool kernels (power-of-two C/8) fwd + bwd vs fp32 torch."""
    from zoo.ops.pool import max_pool2d_nhwc
    x = torch.randn(N, H, W, C, device=gpu).bfloat16()
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p, ceil_mode=ceil)
    xg = x.detach().clone().requires_grad_(True)
    y = max_pool2d_nhwc(xg, (k, k), (s, s), (p, p), ceil_mode=ceil)
    assert y.shape == (N, yr.shape[2], yr.shape[3], C)
    assert torch.equal(y.float(), yr.detach().permute(0, 2, 3, 1))  # max of bf16 values is exact
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert rel(xg.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("n", [10, 1000, 4099])
def test_softmax_rows(gpu, dt, log, n):
    from zoo.ops.nn import softmax
    x = (torch.randn(37, n, device=gpu) * 3).to(dt)
    xr = x.detach().float().clone().requires_grad_(True)
    yr = F.log_softmax(xr, -1) if log else F.softmax(xr, -1)
    xg = x.detach().clone().requires_grad_(True)
    y = softmax(xg, -1, log=log)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert rel(y, yr) < tol
    dy = torch.randn(37, n, device=gpu).to(dt)
    y.backward(dy)
    yr.backward(dy.float())
    assert rel(xg.grad, xr.grad) < (1e-4 if dt == torch.float32 else 3e-2)


def test_softmax_other_dim(gpu):
    from zoo.ops.nn import softmax
    x = torch.randn(4, 7, 5, device=gpu)
    assert rel(softmax(x, 1), F.softmax(x, 1)) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("size", [5, 3])
def test_lrn(gpu, dt, size):
    from zoo.ops.nn import lrn_channels_last
    x = torch.randn(2, 6, 6, 24, device=gpu).to(dt)
    alpha, beta, k = 1e-2, 0.75, 2.0

    def ref(t):
        lo = (size - 1) // 2
        sq = F.pad(t * t, (lo, size - 1 - lo))
        return t * (k + alpha / size * sq.unfold(-1, size, 1).sum(-1)) ** (-beta)
    xr = x.detach().float().clone().requires_grad_(True)
    yr = ref(xr)
    xg = x.detach().clone().requires_grad_(True)
    y = lrn_channels_last(xg, size, alpha, beta, k)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert rel(y, yr) < tol
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    assert rel(xg.grad, xr.grad) < (1e-4 if dt == torch.float32 else 3e-2)
