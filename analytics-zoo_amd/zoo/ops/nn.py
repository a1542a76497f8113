"""LayerNorm and embedding ops on the native kernels (HK12, HK9).

Gradients of parameters re-homed into the engine's flat buffer are added by
the kernels directly (fp32 atomics), exactly like the conv weight gradients.
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native


def _target(p, shape=None):
    g = getattr(p, "_zoo_grad", None)
    if g is not None:
        return g, True
    return torch.zeros(shape if shape is not None else p.shape, dtype=torch.float32, device=p.device), False


def _ready(p):
    h = getattr(p, "_zoo_grad_ready", None)
    if h is not None:
        h(p)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        y, mean, rstd = native().layernorm_fwd(x, None if gamma is None else gamma.detach(),
                                               None if beta is None else beta.detach(), eps)
        ctx.save_for_backward(x, gamma, beta, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mean, rstd = ctx.saved_tensors
        dg, own_g = _target(gamma) if gamma is not None else (None, False)
        db, own_b = _target(beta) if beta is not None else (None, False)
        dx = native().layernorm_bwd(dy.contiguous().to(x.dtype), x, None if gamma is None else gamma.detach(), mean,
                                    rstd, dg, db)
        if own_g:
            _ready(gamma)
        if own_b:
            _ready(beta)
        return dx, (None if own_g else dg), (None if own_b else db), None


_DROP_RNG = []
_DROP_FUSE_MIN = 1 << 22


def _drop_rng():
    if not _DROP_RNG:
        import random
        _DROP_RNG.append(random.Random(torch.initial_seed()))
    return _DROP_RNG[0]


class _DropoutAddFn(torch.autograd.Function):
    """out = x + dropout(a): one native pass; the keep-mask is a counter-based hash of a
    per-call seed, so backward regenerates it (no mask tensor is stored)."""

    @staticmethod
    def forward(ctx, a, x, p):
        seed = _drop_rng().getrandbits(62)   # host RNG: no device sync, no tensor op
        ctx.p, ctx.seed = p, seed
        return native().dropout_add(a, x, p, seed)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        return native().dropout_add(g, None, ctx.p, ctx.seed), g, None


def dropout_add(a, x, p, training=True):
    """``x + F.dropout(a, p, training)`` (Transformer residual branch)."""
    if not training or p <= 0:
        return x + a
    if a.is_cuda and a.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and a.shape == x.shape and \
            a.numel() % 8 == 0 and a.numel() >= _DROP_FUSE_MIN and not torch.cuda.is_current_stream_capturing():
        # small tensors are launch/host-bound: the C++ dropout path has less per-call overhead
        return _DropoutAddFn.apply(a.contiguous(), x.contiguous(), float(p))
    return x + F.dropout(a, p, True)


def layer_norm(x, gamma=None, beta=None, eps=1e-5):
    D = x.shape[-1]
    if x.is_cuda and D % 8 == 0 and x.dtype in (torch.float32, torch.bfloat16):
        return _LayerNormFn.apply(x.contiguous(), gamma, beta, float(eps))
    if (gamma is not None and gamma.dtype != x.dtype) or (beta is not None and beta.dtype != x.dtype):
        # fp32 affine parameters with a low-precision input: normalise in fp32
        return F.layer_norm(x.float(), (D,), None if gamma is None else gamma.float(),
                            None if beta is None else beta.float(), eps).to(x.dtype)
    return F.layer_norm(x, (D,), gamma, beta, eps)


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, idx, pad, compute_dtype):
        src = table
        if compute_dtype is not None and table.dtype != compute_dtype:
            src = getattr(table, "_zoo_bf16", None)
            if src is None or src.dtype != compute_dtype:
                src = table.detach().to(compute_dtype)
        out = native().embedding_fwd(src.contiguous(), idx, pad)
        ctx.save_for_backward(idx)
        ctx.table = table
        ctx.pad = pad
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        table = ctx.table
        g, own = _target(table)
        native().embedding_bwd(dout.contiguous(), idx, g, ctx.pad, 1.0)
        if own:
            _ready(table)
            return None, None, None, None
        return g.to(table.dtype), None, None, None


def embedding(idx, table, padding_idx=None, compute_dtype=None):
    """Row gather ``table[idx]``; backward scatter-adds into the table gradient."""
    idx = idx.long()
    D = table.shape[1]
    dt = compute_dtype or table.dtype
    aligned = (dt == torch.float32 and D % 4 == 0) or (dt == torch.bfloat16 and D % 8 == 0)
    if table.is_cuda and aligned:
        pad = -1 if padding_idx is None else int(padding_idx)
        return _EmbeddingFn.apply(table, idx.contiguous(), pad, compute_dtype)
    out = F.embedding(idx, table, padding_idx=padding_idx)
    return out if compute_dtype is None else out.to(compute_dtype)
