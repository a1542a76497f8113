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
    def forward(ctx, x, R, S, sh, sw, ph, pw):
        y, arg = native().maxpool_fwd(x, R, S, sh, sw, ph, pw, True)
        ctx.save_for_backward(arg)
        ctx.g = (x.shape[1], x.shape[2], R, S, sh, sw, ph, pw)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        H, W, R, S, sh, sw, ph, pw = ctx.g
        dx = native().maxpool_bwd(dy.contiguous().to(torch.bfloat16), arg, H, W, R, S, sh, sw, ph, pw)
        return dx, None, None, None, None, None, None


def max_pool2d_nhwc(x, kernel=(2, 2), stride=None, pad=(0, 0)):
    stride = stride or kernel
    if x.is_cuda and x.shape[-1] % 8 == 0:
        xb = x.to(torch.bfloat16).contiguous()
        y = _MaxPoolFn.apply(xb, kernel[0], kernel[1], stride[0], stride[1], pad[0], pad[1])
        return y if x.dtype == torch.bfloat16 else y.to(x.dtype)
    y = F.max_pool2d(x.permute(0, 3, 1, 2).float(), kernel, stride, pad)
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
