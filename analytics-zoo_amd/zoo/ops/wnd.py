"""Wide & Deep glue ops on native kernels (csrc/kernels/wnd.hip).

``deep_input``: the deep tower's input row -- dense column blocks and per-column embedding
lookups (float ids, the Keras input dtype) concatenated -- built in one kernel straight into the
bf16 MFMA operand; backward scatter-adds into the tables' fp32 (flat) gradients.
``wnd_head``: softmax(wide + bias + deep) in one pass; backward writes both towers' logit
gradients and the bias gradient. Reference: WideAndDeep.scala:113-144 (the deep/wide merge and
the model's final SoftMax). CPU: the plain torch composition.
"""
import torch

from zoo.ops._native import native
from zoo.ops.nn import _ready, _target


class _DeepInputFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, id_cols, *srcs):
        out = native().deep_input_fwd(ids, [s.detach().float().contiguous() for s in srcs], list(id_cols))
        ctx.save_for_backward(ids, *srcs)
        ctx.id_cols = id_cols
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, *srcs = ctx.saved_tensors
        grads, owned, ret = [], [], []
        for s, ic in zip(srcs, ctx.id_cols):
            if ic >= 0 and ctx.needs_input_grad[2 + len(grads)]:
                g, own = _target(s)
                grads.append(g)
                owned.append(own)
            else:
                grads.append(torch.empty(0, device=dout.device))
                owned.append(None)
        native().deep_input_bwd(dout.contiguous().to(torch.bfloat16), ids,
                                [s.detach().float().contiguous() for s in srcs], list(ctx.id_cols), grads)
        for s, ic, g, own in zip(srcs, ctx.id_cols, grads, owned):
            if own is None:
                # dense segments are data inputs; their (rare) gradient is a column slice
                ret.append(None)
            elif own:
                _ready(s)
                ret.append(None)
            else:
                ret.append(g.to(s.dtype))
        if any(ic < 0 and ctx.needs_input_grad[2 + k] for k, ic in enumerate(ctx.id_cols)):
            col = 0
            for k, (s, ic) in enumerate(zip(srcs, ctx.id_cols)):
                w = s.shape[1]
                if ic < 0 and ctx.needs_input_grad[2 + k]:
                    ret[k] = dout[:, col:col + w].to(s.dtype)
                col += w
        return (None, None) + tuple(ret)


def deep_input(ids, segments):
    """``segments``: list of ``("dense", x [B, w])`` or ``("embed", table [V, D], id_column)``;
    returns the concatenated [B, sum(widths)] row (bf16 on the GPU, fp32 on the CPU). Ids are
    zero-based row indices stored as floats in ``ids`` [B, E]; out-of-range ids read zeros."""
    srcs, cols = [], []
    for s in segments:
        if s[0] == "dense":
            srcs.append(s[1])
            cols.append(-1)
        else:
            srcs.append(s[1])
            cols.append(int(s[2]))
    if ids.is_cuda and len(srcs) <= 8 and all(t.dim() == 2 for t in srcs):
        return _DeepInputFn.apply(ids.float().contiguous(), tuple(cols), *srcs)
    parts = []
    for t, c in zip(srcs, cols):
        if c < 0:
            parts.append(t.float())
        else:
            idx = ids[:, c].long()
            ok = (idx >= 0) & (idx < t.shape[0])
            parts.append(t[idx.clamp(0, t.shape[0] - 1)] * ok.unsqueeze(1).to(t.dtype))
    return torch.cat(parts, 1)


class _WndHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wide, deep, bias):
        p = native().wnd_head_fwd(None if wide is None else wide.detach().float().contiguous(),
                                  None if deep is None else deep.detach().contiguous(),
                                  None if bias is None else bias.detach().float().contiguous())
        ctx.save_for_backward(p, bias)
        ctx.has = (wide is not None, deep is not None)
        ctx.deep_dtype = None if deep is None else deep.dtype
        return p

    @staticmethod
    def backward(ctx, g):
        p, bias = ctx.saved_tensors
        gb, own = (None, False)
        if bias is not None and ctx.needs_input_grad[2]:
            gb, own = _target(bias)
        dw, dd = native().wnd_head_bwd(p, g.float().contiguous(), ctx.has[0] and ctx.needs_input_grad[0],
                                       ctx.has[1] and ctx.needs_input_grad[1],
                                       ctx.deep_dtype == torch.bfloat16, gb)
        if gb is not None and own:
            _ready(bias)
            gb = None
        elif gb is not None:
            gb = gb.to(bias.dtype)
        return (dw if dw is not None and dw.numel() else None,
                (dd.to(ctx.deep_dtype) if dd is not None and dd.numel() else None), gb)


def wnd_head(wide=None, deep=None, bias=None):
    """softmax(wide + bias + deep) -> fp32 probabilities [B, C]."""
    ref = wide if wide is not None else deep
    if ref.is_cuda and ref.dim() == 2 and ref.shape[1] <= 32 and \
            (deep is None or deep.dtype in (torch.float32, torch.bfloat16)):
        return _WndHeadFn.apply(wide, None if deep is None else deep.contiguous(), bias)
    z = 0
    if wide is not None:
        z = z + wide.float()
    if bias is not None:
        z = z + bias.float()
    if deep is not None:
        z = z + deep.float()
    return torch.softmax(z, -1)
