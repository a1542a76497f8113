"""Axis reductions and L2-normalisation on the native row kernels (csrc/kernels/reduce.hip,
HK14: AutoGrad.sum / mean / max / min, l2Normalize). The reduced axis is moved last (a
copy only when it is not already last); backward of sum / mean is a broadcast, of max /
min the gradient goes to the (first) extremal element. CPU tensors use torch."""
import torch

from zoo.ops._native import native

_OPS = {"sum": 0, "mean": 1, "max": 2, "min": 3}


def _last(x, axis):
    axis = axis % x.dim()
    return (x if axis == x.dim() - 1 else x.movedim(axis, -1)).contiguous(), axis


class _ReduceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, axis, op, keepdim):
        xl, ax = _last(x if x.dtype in (torch.float32, torch.bfloat16) else x.float(), axis)
        out = native().row_reduce(xl, _OPS[op])
        if op in ("max", "min"):
            ctx.save_for_backward(x, out)
        ctx.shape, ctx.ax, ctx.op, ctx.keep = x.shape, ax, op, keepdim
        out = out.to(x.dtype) if x.is_floating_point() else out
        return out.unsqueeze(ax) if keepdim else out

    @staticmethod
    def backward(ctx, g):
        ax, op = ctx.ax, ctx.op
        gk = g if ctx.keep else g.unsqueeze(ax)
        if op == "sum":
            return gk.expand(ctx.shape).contiguous(), None, None, None
        if op == "mean":
            return (gk / ctx.shape[ax]).expand(ctx.shape).contiguous(), None, None, None
        x, out = ctx.saved_tensors
        hit = (x == out.unsqueeze(ax).to(x.dtype))
        first = hit & (hit.cumsum(ax) == 1)
        return gk.expand(ctx.shape) * first.to(g.dtype), None, None, None


def reduce(x, axis, op="sum", keepdim=False):
    if x.is_cuda and x.dim() >= 1 and x.numel() > 0 and x.is_floating_point():
        return _ReduceFn.apply(x, axis, op, keepdim)
    if op in ("max", "min"):
        return getattr(x, "amax" if op == "max" else "amin")(dim=axis, keepdim=keepdim)
    return getattr(x, op)(dim=axis, keepdim=keepdim)


class _L2NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, axis, eps):
        xl, ax = _last(x, axis)
        y = native().row_l2norm(xl, None, None, eps)
        ctx.save_for_backward(xl, y)
        ctx.ax, ctx.eps, ctx.last = ax, eps, ax == x.dim() - 1
        return y if ctx.last else y.movedim(-1, ax)

    @staticmethod
    def backward(ctx, g):
        xl, y = ctx.saved_tensors
        gl = (g if ctx.last else g.movedim(ctx.ax, -1)).contiguous().to(xl.dtype)
        dx = native().row_l2norm(xl, gl, y, ctx.eps)
        return (dx if ctx.last else dx.movedim(-1, ctx.ax)), None, None


def l2_normalize(x, axis=-1, eps=1e-12):
    """x / sqrt(max(sum(x^2, axis), eps))."""
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.numel() > 0:
        return _L2NormFn.apply(x, axis, float(eps))
    return x / torch.sqrt(torch.clamp((x * x).sum(dim=axis, keepdim=True), min=eps))


__all__ = ["reduce", "l2_normalize"]
