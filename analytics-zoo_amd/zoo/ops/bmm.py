"""Batched matrix product on the native batched-GEMM kernel (csrc/kernels/bmm.hip, HK2):
``bmm(a, b)`` = ``torch.matmul(a, b)`` for a [..., M, K], b [..., K, N] with broadcast
leading dims. Every transpose needed by forward and backward is a strided view handed to
the kernel (no transposed copies); bf16 operands, fp32 accumulation, output in the
input dtype. CPU tensors take ``torch.matmul``."""
import torch

from zoo.ops._native import native


def _flat3(t, batch):
    return t.expand(*batch, *t.shape[-2:]).reshape(-1, *t.shape[-2:])


class _BmmFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        batch = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
        dt = a.dtype
        a3 = _flat3(a.to(torch.bfloat16), batch)
        b3 = _flat3(b.to(torch.bfloat16), batch)
        c = native().bmm_nt(a3, b3.transpose(1, 2), dt == torch.bfloat16)
        ctx.save_for_backward(a3, b3)
        ctx.shapes = (a.shape, b.shape, batch, a.dtype, b.dtype)
        return c.reshape(*batch, a.shape[-2], b.shape[-1]).to(dt)

    @staticmethod
    def backward(ctx, dc):
        a3, b3 = ctx.saved_tensors
        ashape, bshape, batch, adt, bdt = ctx.shapes
        d3 = dc.to(torch.bfloat16).reshape(-1, dc.shape[-2], dc.shape[-1])
        da = db = None
        if ctx.needs_input_grad[0]:
            da = native().bmm_nt(d3, b3, False).reshape(*batch, *ashape[-2:])       # dC B^T
            da = da.sum_to_size(ashape).to(adt)
        if ctx.needs_input_grad[1]:
            db = native().bmm_nt(a3.transpose(1, 2), d3.transpose(1, 2), False)      # A^T dC
            db = db.reshape(*batch, *bshape[-2:]).sum_to_size(bshape).to(bdt)
        return da, db


def bmm(a, b):
    if a.is_cuda and b.is_cuda and a.dim() >= 2 and b.dim() >= 2 and a.is_floating_point():
        return _BmmFn.apply(a, b)
    return torch.matmul(a, b)


__all__ = ["bmm"]
