"""LayerNorm and embedding ops on the native kernels (HK12, HK9).

Gradients of parameters re-homed into the engine's flat buffer are added by
the kernels directly (fp32 atomics), exactly like the conv weight gradients.
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native
from zoo.parallel.flat import grad_slot


def _target(p, shape=None):
    g = grad_slot(p)
    if g is not None:
        return g, True
    return torch.zeros(shape if shape is not None else p.shape, dtype=torch.float32, device=p.device), False


def _ready(p):
    h = getattr(p, "_zoo_grad_ready", None)
    if h is not None:
        h(p)


def _split_fold_ok(x, gamma, own_g, own_b):
    """LayerNorm backward can leave its dgamma / dbeta fold to the weight-gradient side stream:
    engine-owned gradients inside the engine's backward, bf16 rows on the v2 kernel."""
    from zoo.ops import wstream
    D = x.shape[-1]
    return (own_g and own_b and x.is_cuda and x.dtype == torch.bfloat16 and D % 4 == 0 and D <= 1024 and
            gamma.data_ptr() % 16 == 0 and _LN_V2 and wstream.active(x.device))


_LN_V2 = True


def _fold_on_side(part, x, dg, db, gamma, beta):
    from zoo.ops import wstream
    D = x.shape[-1]
    with wstream.wgrad(x.device, part):
        native().layernorm_fold(part, x.numel() // D, D, dg, db)
        _ready(gamma)
        _ready(beta)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, grad_in=None):
        y, mean, rstd = native().layernorm_fwd(x, None if gamma is None else gamma.detach(),
                                               None if beta is None else beta.detach(), eps)
        ctx.save_for_backward(x, gamma, beta, mean, rstd)
        ctx.grad_in = grad_in
        if grad_in is not None:
            grad_in.armed = True   # a residual consumer of y may park its gradient here
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mean, rstd = ctx.saved_tensors
        dg, own_g = _target(gamma) if gamma is not None else (None, False)
        db, own_b = _target(beta) if beta is not None else (None, False)
        dy2 = None
        h = ctx.grad_in
        if h is not None:
            dy2, h.grad = h.grad, None
            if dy2 is not None:
                dy2 = dy2.contiguous().to(x.dtype)
        if gamma is not None and beta is not None and _split_fold_ok(x, gamma, own_g, own_b):
            dx, _, part = native().layernorm_bwd_split(dy.contiguous().to(x.dtype), x, gamma.detach(), mean, rstd,
                                                       dy2, 0.0, 0, False)
            _fold_on_side(part, x, dg, db, gamma, beta)
            return dx, None, None, None, None
        dx = native().layernorm_bwd(dy.contiguous().to(x.dtype), x, None if gamma is None else gamma.detach(), mean,
                                    rstd, dg, db, dy2)
        if own_g:
            _ready(gamma)
        if own_b:
            _ready(beta)
        return dx, (None if own_g else dg), (None if own_b else db), None, None


_DROP_RNG = []
_DROP_FUSE_MIN = 1 << 22


def _drop_rng():
    if not _DROP_RNG:
        import random
        _DROP_RNG.append(random.Random(torch.initial_seed()))
    return _DROP_RNG[0]


class GradAdd:
    """Residual-gradient handoff between the two consumers of a Transformer block input x:
    the first consumer, a linear layer on the library GEMM (``linear(..., grad_add=h)``),
    arms it in forward; the residual ``dropout_add(a, x, ..., grad_add=h)`` then parks its
    x-gradient here in backward instead of returning it, and the linear's backward folds
    it into its data-gradient GEMM (dx = dy W + g, beta = 1) -- no separate gradient-add
    pass over x. Reference: the residual adds of TransformerLayer.scala:129-181."""
    __slots__ = ("armed", "grad")

    def __init__(self):
        self.armed, self.grad = False, None


class GeluLink:
    """GELU-backward handoff between the two linears of a Transformer FFN
    (``m = linear(n, W1, b1, act="gelu", gelu_link=l); out = linear(m, W2, b2, gelu_src=l)``):
    the first parks its bf16 pre-activation here in forward; the second's backward runs its
    data-gradient GEMM with the GELU derivative applied in the epilogue (and the first's bias
    gradient as the epilogue's column sums), so it returns d pre instead of d m and the first
    skips its activation-backward pass. Valid because m has no other consumer in the block.
    Reference: the FFN of TransformerLayer.scala:129-181."""
    __slots__ = ("pre", "y", "db", "done")

    def __init__(self):
        self.pre = self.y = self.db = None
        self.done = False


def _native_drop(a):
    """The fused native dropout kernels draw their masks from a host seed per call. Eager: for
    tensors of at least _DROP_FUSE_MIN elements. Under hipGraph capture the host seed would be
    baked into the graph, so only once the engine registered the per-step device seed offset the
    kernels xor in (zoo.ops.devscalar) -- then always, so every mask of the captured step follows
    that offset (torch's own dropout would advance its generator per replay instead)."""
    if torch.cuda.is_current_stream_capturing():
        from zoo.ops.devscalar import seed_offset_live
        return seed_offset_live(a.device)
    return a.numel() >= _DROP_FUSE_MIN


class _DropoutAddFn(torch.autograd.Function):
    """out = x + dropout(a): one native pass; the keep-mask is a counter-based hash of a
    per-call seed, so backward regenerates it (no mask tensor is stored)."""

    @staticmethod
    def forward(ctx, a, x, p, handoff=None):
        seed = _drop_rng().getrandbits(62)   # host RNG: no device sync, no tensor op
        ctx.p, ctx.seed = p, seed
        ctx.handoff = handoff if (handoff is not None and handoff.armed) else None
        if ctx.handoff is not None:
            handoff.armed = False   # one parking consumer per arming; any other consumer returns its grad
        return native().dropout_add(a, x, p, seed)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        da = native().dropout_add(g, None, ctx.p, ctx.seed)
        if ctx.handoff is not None:
            h = ctx.handoff           # added by the armed consumer's backward (dgrad GEMM / LayerNorm)
            h.grad = g if h.grad is None else h.grad + g
            return da, None, None, None
        return da, g, None, None


def dropout_add(a, x, p, training=True, grad_add=None):
    """``x + F.dropout(a, p, training)`` (Transformer residual branch). ``grad_add``: a
    :class:`GradAdd` armed by the linear layer that also consumes ``x``."""
    if not training or p <= 0:
        return x + a
    if a.is_cuda and a.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and a.shape == x.shape and \
            a.numel() % 8 == 0 and _native_drop(a):
        # small eager tensors are launch/host-bound: the C++ dropout path has less per-call overhead
        return _DropoutAddFn.apply(a.contiguous(), x.contiguous(), float(p), grad_add)
    return x + F.dropout(a, p, True)


class _DropAddLNFn(torch.autograd.Function):
    """y = LayerNorm(x + dropout(a)) in one native pass (the Transformer residual LayerNorm):
    the residual sum s is formed in registers, stored once for the backward and normalised
    without being read back. Backward: one LayerNorm-backward kernel writes ds and, with the
    regenerated mask, da = keep * ds / (1 - p); ds is x's gradient (or parked in an armed GradAdd)."""

    @staticmethod
    def forward(ctx, a, x, gamma, beta, eps, p, handoff=None, grad_in=None):
        seed = _drop_rng().getrandbits(62)
        y, s, mean, rstd = native().dropout_add_layernorm_fwd(a, x, gamma.detach(), beta.detach(), eps, p, seed)
        ctx.save_for_backward(s, gamma, beta, mean, rstd)
        ctx.p, ctx.seed = p, seed
        ctx.handoff = handoff if (handoff is not None and handoff.armed) else None
        if ctx.handoff is not None:
            handoff.armed = False   # one parking consumer per arming, as _DropoutAddFn
        ctx.grad_in = grad_in
        if grad_in is not None:
            grad_in.armed = True
        return y

    @staticmethod
    def backward(ctx, dy):
        s, gamma, beta, mean, rstd = ctx.saved_tensors
        dg, own_g = _target(gamma)
        db, own_b = _target(beta)
        dy2 = None
        h = ctx.grad_in
        if h is not None:
            dy2, h.grad = h.grad, None
            if dy2 is not None:
                dy2 = dy2.contiguous().to(s.dtype)
        # one kernel writes ds and the dropout branch's da = keep * ds / (1 - p); the dgamma / dbeta
        # fold goes to the weight-gradient side stream when the engine owns those gradients
        if _split_fold_ok(s, gamma, own_g, own_b):
            ds, da, part = native().layernorm_bwd_split(dy.contiguous().to(s.dtype), s, gamma.detach(), mean, rstd,
                                                        dy2, ctx.p, ctx.seed, True)
            _fold_on_side(part, s, dg, db, gamma, beta)
        else:
            ds, da = native().layernorm_bwd_drop(dy.contiguous().to(s.dtype), s, gamma.detach(), mean, rstd, dg, db,
                                                 dy2, ctx.p, ctx.seed)
            if own_g:
                _ready(gamma)
            if own_b:
                _ready(beta)
        dx = ds
        if ctx.handoff is not None:
            hh = ctx.handoff
            hh.grad = ds if hh.grad is None else hh.grad + ds
            dx = None
        return da, dx, (None if own_g else dg), (None if own_b else db), None, None, None, None


def dropout_add_layer_norm(a, x, p, training, gamma, beta, eps=1e-5, grad_add=None, grad_in=None):
    """``layer_norm(dropout_add(a, x, p, training, grad_add), gamma, beta, eps, grad_in)`` -- the
    Transformer residual LayerNorm -- as one native pass when it can be (bf16 GPU tensors, fp32
    affine, D % 8 == 0, D <= 2048, dropout live, ``_native_drop``: the mask seed is drawn on the
    host per call); otherwise the two ops. Reference: TransformerLayer.scala:129-181."""
    D = x.shape[-1]
    if training and p > 0 and a.is_cuda and a.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and \
            a.shape == x.shape and D % 8 == 0 and D <= 2048 and a.numel() >= _DROP_FUSE_MIN and \
            gamma is not None and beta is not None and gamma.dtype == torch.float32 and \
            beta.dtype == torch.float32 and _native_drop(a):
        return _DropAddLNFn.apply(a.contiguous(), x.contiguous(), gamma, beta, float(eps), float(p), grad_add, grad_in)
    return layer_norm(dropout_add(a, x, p, training, grad_add=grad_add), gamma, beta, eps, grad_in=grad_in)


def layer_norm(x, gamma=None, beta=None, eps=1e-5, grad_in=None):
    """``grad_in``: a :class:`GradAdd` the consumers of the OUTPUT can park a gradient in
    (``dropout_add(a, y, ..., grad_add=h)``, the Transformer residual): the backward kernel sums
    it with the incoming gradient, so autograd runs no separate add over y."""
    D = x.shape[-1]
    if x.is_cuda and D % 8 == 0 and x.dtype in (torch.float32, torch.bfloat16):
        return _LayerNormFn.apply(x.contiguous(), gamma, beta, float(eps), grad_in)
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
            else:
                table._zoo_bf16_read = True
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
    if getattr(table, "_zoo_row_sparse", False):
        from zoo.parallel.ddp import record_lookup
        record_lookup(table, idx)
    D = table.shape[1]
    dt = compute_dtype or table.dtype
    aligned = (dt == torch.float32 and D % 4 == 0) or (dt == torch.bfloat16 and D % 8 == 0)
    if table.is_cuda and aligned:
        pad = -1 if padding_idx is None else int(padding_idx)
        return _EmbeddingFn.apply(table, idx.contiguous(), pad, compute_dtype)
    out = F.embedding(idx, table, padding_idx=padding_idx)
    return out if compute_dtype is None else out.to(compute_dtype)


# ---------------------------------------------------------------------------
# depthwise convolution (NHWC bf16, tap-major weight [R*S, C])
# ---------------------------------------------------------------------------
class _DwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, R, S, stride, pad, act):
        from zoo.ops.conv import bf16_weight
        C_ = native()
        wb = bf16_weight(w).contiguous()
        y = C_.dwconv_fwd(x, wb, None if bias is None else bias.detach().float().contiguous(), R, S, stride[0],
                          stride[1], pad[0], pad[1], _ACT.get(act, 0))
        ctx.save_for_backward(x, w, y if act == "relu" else None)
        ctx.g = (R, S, stride, pad, act, bias is not None, x.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        C_ = native()
        x, w, y = ctx.saved_tensors
        R, S, stride, pad, act, has_bias, xs = ctx.g
        dy = dy.contiguous().to(torch.bfloat16)
        if act == "relu":
            dy = dy * (y > 0).to(dy.dtype)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            from zoo.ops.conv import bf16_weight
            dx = C_.dwconv_dgrad(dy, bf16_weight(w).contiguous(), xs[1], xs[2], R, S, stride[0], stride[1], pad[0],
                                 pad[1])
        if ctx.needs_input_grad[1]:
            tgt, own = _target(w)
            C_.dwconv_wgrad(x, dy, tgt, R, S, stride[0], stride[1], pad[0], pad[1])
            if own:
                _ready(w)
            else:
                dw = tgt.to(w.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().reshape(-1, dy.shape[-1]).sum(0)
        return dx, dw, db, None, None, None, None, None


_ACT = {None: 0, "linear": 0, "relu": 1, "gelu": 2, "sigmoid": 3, "tanh": 4}


def depthwise_bn_act_eval(x, w, gamma, beta, running_mean, running_var, kernel, stride, pad, eps=1e-5, relu=True):
    """Eval-mode depthwise conv -> BN(running stats) -> ReLU as one kernel (BN folded into
    the per-channel taps and a bias)."""
    from zoo.ops.bn import _folded
    wf, bf = _folded(w, gamma, beta, running_mean, running_var, eps, cols=True)
    return native().dwconv_fwd(x.to(torch.bfloat16).contiguous(), wf, bf, kernel[0], kernel[1], stride[0], stride[1],
                               pad[0], pad[1], 1 if relu else 0)


def depthwise_conv2d_nhwc(x, w, bias=None, kernel=(3, 3), stride=(1, 1), pad=(0, 0), act=None):
    """Depthwise conv, x [N,H,W,C], w [R*S, C] (tap-major), optional fused bias + relu."""
    R, S = kernel
    C = x.shape[-1]
    if x.is_cuda and C % 8 == 0 and R * S <= 9 and act in (None, "linear", "relu"):
        return _DwConvFn.apply(x.to(torch.bfloat16).contiguous(), w, bias, R, S, tuple(stride), tuple(pad), act)
    wt = w.float().t().reshape(C, 1, R, S)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), wt, None if bias is None else bias.float(), stride, pad, groups=C)
    if act in (None, "linear"):
        from zoo.ops.conv import ref_storage
        y = ref_storage(y)     # stored in bf16 on the GPU before the BatchNorm that follows
    if act == "relu":
        y = torch.relu(y)
    elif act not in (None, "linear"):
        y = getattr(torch, act)(y)
    return y.permute(0, 2, 3, 1).to(x.dtype)


# ---------------------------------------------------------------------------
# row softmax / log-softmax (last dim)
# ---------------------------------------------------------------------------
class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, log_out):
        y = native().softmax_rows(x, log_out)
        ctx.save_for_backward(y)
        ctx.log_out = log_out
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return native().softmax_rows_bwd(y, dy.contiguous().to(y.dtype), ctx.log_out), None


def softmax(x, dim=-1, log=False):
    """Softmax / LogSoftmax over ``dim`` on the native row kernel (fp32 or bf16)."""
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.numel() > 0:
        moved = dim not in (-1, x.dim() - 1)
        xt = x.movedim(dim, -1) if moved else x
        y = _SoftmaxFn.apply(xt.contiguous(), bool(log))
        return y.movedim(-1, dim) if moved else y
    return F.log_softmax(x, dim) if log else F.softmax(x, dim)


# ---------------------------------------------------------------------------
# cross-channel LRN (channels last)
# ---------------------------------------------------------------------------
class _LRNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, alpha, beta, k):
        ctx.save_for_backward(x)
        ctx.p = (size, alpha, beta, k)
        return native().lrn(x, None, size, alpha, beta, k)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        size, alpha, beta, k = ctx.p
        return native().lrn(x, dy.contiguous().to(x.dtype), size, alpha, beta, k), None, None, None, None


def lrn_channels_last(x, size=5, alpha=1e-4, beta=0.75, k=1.0):
    """y = x * (k + alpha/size * sum_{window} x^2)^-beta over the LAST dim (BigDL
    SpatialCrossMapLRN semantics; the window is centred, (size-1)/2 below)."""
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.numel() > 0:
        return _LRNFn.apply(x.contiguous(), int(size), float(alpha), float(beta), float(k))
    xc = x.float()
    lo = (size - 1) // 2
    sq = F.pad((xc * xc).unsqueeze(1), (lo, size - 1 - lo)).squeeze(1)
    s = sq.unfold(-1, size, 1).sum(-1)
    return (xc * (k + alpha / size * s) ** (-beta)).to(x.dtype)
