"""NHWC pooling ops (max with byte-argmax for a gather-form backward, global average).

Reference: BigDL SpatialMaxPooling / SpatialAveragePooling behind the Keras
pooling layers (Zs/pipeline/api/keras/layers/MaxPooling2D.scala,
GlobalAveragePooling2D.scala).
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, R, S, sh, sw, ph, pw, ceil_mode=False):
        y, arg = native().maxpool_fwd(x, R, S, sh, sw, ph, pw, True, bool(ceil_mode))
        ctx.save_for_backward(arg)
        ctx.g = (x.shape[1], x.shape[2], R, S, sh, sw, ph, pw)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        H, W, R, S, sh, sw, ph, pw = ctx.g
        dx = native().maxpool_bwd(dy.contiguous().to(torch.bfloat16), arg, H, W, R, S, sh, sw, ph, pw)
        return dx, None, None, None, None, None, None, None


def max_pool2d_nhwc(x, kernel=(2, 2), stride=None, pad=(0, 0), ceil_mode=False):
    stride = stride or kernel
    if x.is_cuda and x.shape[-1] % 8 == 0:
        xb = x.to(torch.bfloat16).contiguous()
        y = _MaxPoolFn.apply(xb, kernel[0], kernel[1], stride[0], stride[1], pad[0], pad[1], ceil_mode)
        return y if x.dtype == torch.bfloat16 else y.to(x.dtype)
    y = F.max_pool2d(x.permute(0, 3, 1, 2).float(), kernel, stride, pad, ceil_mode=ceil_mode)
    return y.permute(0, 2, 3, 1).to(x.dtype)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, R, S, sh, sw, ph, pw, ceil_mode, inc_pad):
        ctx.g = (x.shape[1], x.shape[2], R, S, sh, sw, ph, pw, inc_pad)
        return native().avgpool_fwd(x, R, S, sh, sw, ph, pw, ceil_mode, inc_pad)

    @staticmethod
    def backward(ctx, dy):
        H, W, R, S, sh, sw, ph, pw, inc_pad = ctx.g
        dx = native().avgpool_bwd(dy.contiguous().to(torch.bfloat16), H, W, R, S, sh, sw, ph, pw, inc_pad)
        return dx, None, None, None, None, None, None, None, None


def avg_pool2d_nhwc(x, kernel=(2, 2), stride=None, pad=(0, 0), ceil_mode=False, count_include_pad=True):
    """NHWC average pooling (AveragePooling2D / SpatialAveragePooling)."""
    stride = stride or kernel
    if x.is_cuda and x.shape[-1] % 8 == 0 and 2 * pad[0] <= kernel[0] and 2 * pad[1] <= kernel[1]:
        xb = x.to(torch.bfloat16).contiguous()
        y = _AvgPoolFn.apply(xb, kernel[0], kernel[1], stride[0], stride[1], pad[0], pad[1], bool(ceil_mode),
                             bool(count_include_pad))
        return y if x.dtype == torch.bfloat16 else y.to(x.dtype)
    y = F.avg_pool2d(x.permute(0, 3, 1, 2).float(), kernel, stride, pad, ceil_mode=ceil_mode,
                     count_include_pad=count_include_pad)
    return y.permute(0, 2, 3, 1).to(x.dtype)


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return native().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return native().gap_bwd(dy.contiguous().to(torch.bfloat16), ctx.hw[0], ctx.hw[1])


def global_avg_pool_nhwc(x):
    if x.is_cuda and x.shape[-1] % 8 == 0:
        xb = x.to(torch.bfloat16).contiguous()
        y = _GapFn.apply(xb)
        return y if x.dtype == torch.bfloat16 else y.to(x.dtype)
    return x.float().mean(dim=(1, 2)).to(x.dtype)
