"""Fused NeuralCF step (csrc/kernels/ncf.hip): the whole NCF network -- embedding gathers, MLP
tower, matrix-factorisation product, concat, Dense + softmax -- as one native kernel per
direction, with the weight gradients on the matrix cores and the embedding-row gradients
scattered straight into the (flat) gradient buffers.

Reference: NeuralCF.scala:45-138 (Zs/models/recommendation), Py models/recommendation/neuralcf.py.
``ncf_reference`` is the plain fp32 PyTorch twin of the same computation (CPU tests / parity).
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native
from zoo.parallel.flat import grad_slot


def _t(p):
    return p if p is not None else None


def _empty(dev):
    return torch.empty(0, device=dev)


def _grad_target(p):
    g = grad_slot(p)
    if g is not None:
        return g, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), False


def _ready(p):
    h = getattr(p, "_zoo_grad_ready", None)
    if h is not None:
        h(p)


def _table_src(tables):
    """bf16 engine copies of the four tables when every one has one, else the fp32 tables."""
    copies = [getattr(t, "_zoo_bf16", None) if t is not None else None for t in tables]
    if all(c is not None and c.dtype == torch.bfloat16 for c, t in zip(copies, tables) if t is not None):
        for t in tables:
            if t is not None:
                t._zoo_bf16_read = True
        return [c if t is not None else None for c, t in zip(copies, tables)]
    return [t.detach() if t is not None else None for t in tables]


class _NcfFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, dims, *params):
        # params: tu, ti, tmu, tmi, w1, b1, w2, b2, w3, b3, wo, bo (None = absent)
        dev = ids.device
        tabs = _table_src(params[:4])
        ts = [x.contiguous() if x is not None else _empty(dev) for x in tabs]
        ws = [p.detach().float().contiguous() if p is not None else _empty(dev) for p in params[4:]]
        probs = native().ncf_fused(ids, ts + ws, list(dims), None, [])
        ctx.save_for_backward(ids, probs)
        ctx.dims, ctx.params, ctx.ts, ctx.ws = dims, params, ts, ws
        return probs

    @staticmethod
    def backward(ctx, dprobs):
        ids, _ = ctx.saved_tensors
        params = ctx.params
        targets = []
        for p in params:
            if p is None or not p.requires_grad:
                targets.append(None)
            else:
                targets.append(_grad_target(p))
        dev = ids.device
        g = [tg[0] if tg is not None else _empty(dev) for tg in targets]
        native().ncf_fused(ids, ctx.ts + ctx.ws, list(ctx.dims), dprobs.float().contiguous(), g)
        out = []
        for p, tg in zip(params, targets):
            if tg is None:
                out.append(None)
            elif tg[1]:
                _ready(p)
                out.append(None)
            else:
                out.append(tg[0].to(p.dtype))
        ctx.ts = ctx.ws = ctx.params = None
        return (None, None) + tuple(out)


def ncf_fused_ok(dims):
    """dims = (eu, ei, em, h1, h2, h3, nc, id_off): the native kernel covers these widths."""
    try:
        return native().ncf_tier(list(dims)) >= 0
    except Exception:  # noqa: BLE001
        return False


def ncf_fused(ids, dims, tu, ti, tmu, tmi, w1, b1, w2, b2, w3, b3, wo, bo):
    """probs [B, nc] (fp32) of the NeuralCF network for ``ids`` [B, 2] (user, item)."""
    return _NcfFn.apply(ids.long().contiguous(), tuple(int(d) for d in dims), tu, ti, tmu, tmi, w1, b1, w2, b2,
                        w3, b3, wo, bo)


class _Bf16Stage(torch.autograd.Function):
    """Round to bf16 in the forward AND the backward: the kernel parks activations and staged
    gradients as bf16 LDS rows (csrc/kernels/ncf.hip), this replays that rounding in fp32."""

    @staticmethod
    def forward(ctx, x):
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def ncf_reference(ids, tu, ti, tmu, tmi, w1, b1, w2, b2, w3, b3, wo, bo, id_off=0, bf16_stage=False):
    """Plain fp32 PyTorch NeuralCF forward (same math as the kernel; CPU / parity tests).
    ``bf16_stage``: round at the points where the kernel stages through bf16 (gathered rows,
    hidden activations and their pre-activation gradients) -- the
    emulated-bf16 baseline the kernel's gradient noise is measured against."""
    st = _Bf16Stage.apply if bf16_stage else (lambda t: t)
    u = ids[:, 0].long() - id_off
    i = ids[:, 1].long() - id_off
    h = st(torch.cat([F.embedding(u, tu.float()), F.embedding(i, ti.float())], 1))
    for w, b in ((w1, b1), (w2, b2), (w3, b3)):
        h = torch.relu(st(F.linear(h, w.float(), None if b is None else b.float())))
    if tmu is not None:
        h = torch.cat([h, st(F.embedding(u, tmu.float()) * F.embedding(i, tmi.float()))], 1)
    return torch.softmax(F.linear(h, wo.float(), None if bo is None else bo.float()), -1)
