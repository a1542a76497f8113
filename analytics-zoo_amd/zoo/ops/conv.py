"""NHWC convolution / linear ops on the gfx950 implicit-GEMM kernels.

Weights are kept in the native *packed* layout ``[K, ldb]`` where a row is the
logical ``[R][S][C]`` filter flattened and zero padded to ``ldb = ceil8(R*S*C)``
(16-byte aligned rows for the MFMA B-operand loads). The fp32 master weight and
its bf16 compute copy both use this layout, so the fused optimizer can update
master + copy in one pass over flat buffers.

Backward:
  * dX  = transposed conv of dY with flipped weights (``flip_weights`` + igemm
    with input dilation = stride)
  * dW += wgrad(X, dY) accumulated in fp32 straight into the parameter's
    gradient (``param._zoo_grad`` when the engine owns a flat gradient buffer).

Reference: BigDL SpatialConvolution / Linear behind
Zs/pipeline/api/keras/layers/Convolution2D.scala:86-110 and Dense.scala:97
(SURVEY.md §2.16 HK1/HK3/HK5).
"""
import math
import os

import torch
import torch.nn.functional as F

from zoo.ops._native import native
from zoo.ops import _kern, wstream
from zoo.parallel.flat import grad_slot

# training GELU linears: pre-activation stored by the GEMM epilogue beside the output (False: the
# GEMM writes v and a separate GELU pass forms the output -- the oracle / A/B of round 6)
_GELU_DUAL = True
ACT_CODES = {None: 0, "linear": 0, "relu": 1, "gelu": 2, "sigmoid": 3, "tanh": 4}


def ceil8(v):
    return (v + 7) // 8 * 8


def conv_out_size(h, r, stride, pad, dil=1):
    return (h + 2 * pad - dil * (r - 1) - 1) // stride + 1


def bf16_weight(w):
    """bf16 compute copy of a packed weight: engine-maintained (``_zoo_bf16``, a
    view into the flat bf16 buffer the optimizer rewrites) when training;
    otherwise converted once and cached on the parameter until it is modified
    (in-place updates bump ``_version``), so inference pays no per-call cast."""
    c = getattr(w, "_zoo_bf16", None)
    if c is not None:
        w._zoo_bf16_read = True   # ZeRO-1 may gather this parameter as bf16 (parallel/ddp.py)
        return c
    if w.dtype == torch.bfloat16:
        return w.detach()
    cc = getattr(w, "_zoo_bf16_cache", None)
    if cc is not None and cc[0] == w._version and cc[1] == w.data_ptr():
        return cc[2]
    b = w.detach().to(torch.bfloat16)
    if not torch.is_grad_enabled() or not w.requires_grad:
        try:
            w._zoo_bf16_cache = (w._version, w.data_ptr(), b)
        except (AttributeError, RuntimeError):
            pass
    return b


def accumulate_grad(param, g):
    """Return the gradient autograd should accumulate, or None if the kernel
    already accumulated into the engine-owned flat gradient buffer."""
    return g


def _ref_act(y, act):
    if act in (None, "linear"):
        return y
    if act == "relu":
        return torch.relu(y)
    if act == "gelu":
        return F.gelu(y)
    if act == "sigmoid":
        return torch.sigmoid(y)
    if act == "tanh":
        return torch.tanh(y)
    raise ValueError(act)


def unpack_weight(w2, K, R, S, C):
    return w2[:, : R * S * C].reshape(K, R, S, C)


def pack_weight(w4):
    K, R, S, C = w4.shape
    ldb = ceil8(R * S * C)
    out = torch.zeros(K, ldb, dtype=w4.dtype, device=w4.device)
    out[:, : R * S * C] = w4.reshape(K, R * S * C)
    return out


# Parity harness switch (tools/layer_parity.py): the CPU reference then rounds a conv output that the
# GPU path stores in bf16 before a BatchNorm reads it (conv -> BN units), so the reference and the
# kernels see the same pre-activations and a ReLU mask does not flip on that rounding alone.
REF_BF16_STORAGE = [False]


def ref_storage(y):
    """``y`` rounded to bf16 and back when the parity harness emulates bf16 storage."""
    return y.to(torch.bfloat16).float() if REF_BF16_STORAGE[0] else y


# Parity harness switch for the BACKWARD comparison: [keep-mask, uses]. A pre-activation that lands
# within rounding of zero is a tie -- either ReLU decision is correct -- but a tie decided
# differently by the GPU and the CPU twin moves that element's whole gradient. With a mask set,
# the CPU paths' ReLU keeps exactly the elements the GPU forward kept (the forward itself is
# compared without it) and counts its uses, so the harness can check it hit one ReLU.
REF_RELU_MASK = [None, 0]


def ref_relu(z):
    m = REF_RELU_MASK[0]
    if m is not None and m.shape == z.shape:
        REF_RELU_MASK[1] += 1
        return z * m.to(z.dtype)
    return torch.relu(z)


def conv2d_ref(x, w2, geom, bias=None):
    """fp32 PyTorch reference: x NHWC, packed weight -> NHWC."""
    R, S, C, stride, pad, dil = geom
    K = w2.shape[0]
    w4 = unpack_weight(w2.float(), K, R, S, C).permute(0, 3, 1, 2)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w4, bias=None if bias is None else bias.float(), stride=stride,
                 padding=pad, dilation=dil)
    return y.permute(0, 2, 3, 1)


class _Conv2dFn(torch.autograd.Function):
    """y = act(conv(x, w) + b) on NHWC bf16 with the native kernels."""

    @staticmethod
    def forward(ctx, x, w, bias, R, S, stride, pad, dil, act, out_f32):
        ctx.bias_ref = bias
        wb = bf16_weight(w)
        y = _kern.conv_fwd(x, wb, R, S, stride, pad, dil, bias=None if bias is None else bias.detach().float().contiguous(),
                           act=ACT_CODES[act], out_f32=out_f32, out_bf16=not out_f32)
        ctx.save_for_backward(x, w, y if act not in (None, "linear") else None)
        ctx.geom = (R, S, stride, pad, dil, act, x.shape, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        C_ = native()
        x, w, y = ctx.saved_tensors
        R, S, stride, pad, dil, act, xshape, has_bias = ctx.geom
        dy = dy.contiguous()
        db_native = None
        K = w.shape[0]
        want_db = bool(has_bias and ctx.needs_input_grad[2])
        if K % 8 == 0 and dy.is_cuda and ((act == "relu" and y.dtype == torch.bfloat16) or
                                          (act in (None, "linear") and want_db)):
            # ReLU mask + bias-gradient column sums in one native pass
            # the bias gradient goes straight into the engine's flat gradient buffer when there is one
            bref = getattr(ctx, "bias_ref", None)
            into = grad_slot(bref) if (want_db and bref is not None) else None
            into = into if (into is not None and into.is_contiguous() and into.numel() == K) else None
            outs = C_.act_bwd_reduce(dy.to(torch.bfloat16).contiguous(), y if act == "relu" else None, want_db, into)
            dy = outs[0]
            db_native = outs[1] if len(outs) > 1 else None
            if into is not None:
                hook = getattr(bref, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(bref)
                db_native = "flat"
        elif act == "relu":
            dy = dy * (y > 0).to(dy.dtype)
        elif act not in (None, "linear"):
            yf = y.float()
            if act == "sigmoid":
                dy = dy * (yf * (1 - yf)).to(dy.dtype)
            elif act == "tanh":
                dy = dy * (1 - yf * yf).to(dy.dtype)
            else:
                raise NotImplementedError("backward through fused %s epilogue" % act)
        dyb = dy.to(torch.bfloat16).contiguous()
        K = w.shape[0]
        Cin = xshape[3]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _kern.conv_dgrad(dyb, bf16_weight(w), K, R, S, Cin, xshape[1], xshape[2], stride, pad, dil,
                                  resid=getattr(ctx, "grad_add", None))
        if ctx.needs_input_grad[1]:
            gbuf = grad_slot(w)
            target = gbuf if gbuf is not None else torch.zeros(w.shape, dtype=torch.float32, device=w.device)
            C_.conv_wgrad(x, dyb, target, R, S, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1])
            if gbuf is None:
                dw = target.to(w.dtype)
            else:
                hook = getattr(w, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(w)
        if has_bias and ctx.needs_input_grad[2] and db_native is not None:
            db = None if isinstance(db_native, str) else db_native
        elif has_bias and ctx.needs_input_grad[2]:
            if K % 8 == 0:  # native channel reduction (16-byte loads, ~1024 blocks) instead of torch's sum
                st = torch.zeros(C_.stat_len(K), dtype=torch.float32, device=dyb.device)  # slotted atomics
                C_.bn_reduce(dyb, None, None, None, None, st, 0)
                db = st[:K]
            else:
                db = dy.float().reshape(-1, K).sum(0)
        return dx, dw, db, None, None, None, None, None, None, None


def conv2d_nhwc(x, w, bias=None, kernel=(1, 1), stride=(1, 1), pad=(0, 0), dil=(1, 1), act=None, out_f32=False):
    """NHWC conv with a packed weight [K, ldb]. x: [N,H,W,C]."""
    R, S = kernel
    Cin = x.shape[3]
    if x.is_cuda:
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        if act == "gelu" and torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or
                                                          (bias is not None and bias.requires_grad)):
            # GELU's derivative needs the pre-activation, which the fused epilogue does not keep:
            # training runs the GEMM with a plain epilogue and GELU as a separate op
            y = _Conv2dFn.apply(x.contiguous(), w, bias, R, S, tuple(stride), tuple(pad), tuple(dil), None, out_f32)
            return F.gelu(y)
        return _Conv2dFn.apply(x.contiguous(), w, bias, R, S, tuple(stride), tuple(pad), tuple(dil), act, out_f32)
    y = conv2d_ref(x, w, (R, S, Cin, tuple(stride), tuple(pad), tuple(dil)), bias)
    y = _ref_act(y, act)
    return y if out_f32 or x.dtype == torch.float32 else y.to(x.dtype)


class _GroupedConv2dFn(torch.autograd.Function):
    """y = act(grouped_conv(x, w) + b): every direction is ONE native launch with the group index
    in the grid (csrc/kernels/gconv.hip), no per-group slices / pads / concatenation."""

    @staticmethod
    def forward(ctx, x, w, bias, groups, R, S, stride, pad, dil, act):
        wb = bf16_weight(w)
        y = native().gconv_fwd(x, wb, None if bias is None else bias.detach().float().contiguous(), groups, R, S,
                               stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], ACT_CODES[act])
        ctx.save_for_backward(x, w, y if act not in (None, "linear") else None)
        ctx.geom = (groups, R, S, stride, pad, dil, act, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        groups, R, S, stride, pad, dil, act, has_bias = ctx.geom
        dy = dy.float()
        if act == "relu":
            dy = dy * (y > 0).float()
        elif act == "sigmoid":
            yf = y.float()
            dy = dy * yf * (1 - yf)
        elif act == "tanh":
            yf = y.float()
            dy = dy * (1 - yf * yf)
        elif act not in (None, "linear"):
            raise NotImplementedError("backward through fused %s epilogue" % act)
        dyb = dy.to(torch.bfloat16).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = native().gconv_dgrad(dyb, bf16_weight(w), groups, x.shape[1], x.shape[2], x.shape[3], R, S,
                                      stride[0], stride[1], pad[0], pad[1], dil[0], dil[1])
        if ctx.needs_input_grad[1]:
            gbuf = grad_slot(w)
            target = gbuf if gbuf is not None else torch.zeros(w.shape, dtype=torch.float32, device=w.device)
            native().gconv_wgrad(x, dyb, target, groups, R, S, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1])
            if gbuf is None:
                dw = target.to(w.dtype)
            else:
                hook = getattr(w, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(w)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0)
        return dx, dw, db, None, None, None, None, None, None, None


def grouped_conv2d_nhwc(x, w, bias=None, groups=1, kernel=(1, 1), stride=(1, 1), pad=(0, 0), dil=(1, 1), act=None):
    """Grouped NHWC conv. x: [N, H, W, C] (C = groups * Cg, unpadded); w: packed [K, ldb] where
    row k holds output channel k's filter over its group's (r, s, c), c < Cg (ldb >= R*S*Cg, % 8)."""
    R, S = kernel
    if x.is_cuda:
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        return _GroupedConv2dFn.apply(x.contiguous(), w, bias, int(groups), R, S, tuple(stride), tuple(pad),
                                      tuple(dil), act)
    K = w.shape[0]
    Cg = x.shape[3] // groups
    w4 = w[:, :R * S * Cg].float().reshape(K, R, S, Cg).permute(0, 3, 1, 2)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w4, bias=None if bias is None else bias.float(), stride=stride,
                 padding=pad, dilation=dil, groups=groups).permute(0, 2, 3, 1)
    y = _ref_act(y, act)
    return y if x.dtype == torch.float32 else y.to(x.dtype)


# hipBLASLt for transformer-size linears is an opt-in comparator since round 3 (ZOO_LINEAR_BLAS=1);
# by default they run on the hand-written MFMA GEMMs (_LinearNativeFn)
_BLAS_LINEAR = os.environ.get("ZOO_LINEAR_BLAS", "0") == "1"


class _LinearBlasFn(torch.autograd.Function):
    """Plain (bias / ReLU / GELU) linear layers at transformer sizes on hipBLASLt
    (bf16 in, fp32 accumulate; bias+activation in the library epilogue). On
    MI355X it runs these large plain GEMMs ~1.7x faster than the implicit-GEMM
    kernel (tools/gemm_bench.py --bert), which stays in charge wherever its
    fused epilogues matter (BN statistics, parity dgrad, small/odd shapes).
    Weight gradients accumulate in fp32 into the engine's flat gradient buffer."""

    @staticmethod
    def forward(ctx, x2, w, bias, act, need_grad, grad_add=None):
        ctx.grad_add = grad_add
        if grad_add is not None and need_grad:
            grad_add.armed = True   # the residual consumer of x may now hand its gradient here
        wb = bf16_weight(w)
        bb = None if bias is None else _bf16_bias(bias)
        pre = None
        if act == "gelu" and need_grad:
            pre = torch.addmm(bb, x2, wb.t()) if bb is not None else torch.mm(x2, wb.t())
            # GELU on the native pointwise kernel; the pre-activation is kept for the fused
            # GELU-backward + bias-gradient pass (act_bwd_reduce)
            y = native().act_fwd_bwd(pre, None, 4, 0.0) if pre.is_contiguous() else F.gelu(pre)
        elif act in ("gelu", "relu") and bb is not None:
            y = torch._addmm_activation(bb, x2, wb.t(), use_gelu=(act == "gelu"))
        else:
            y = torch.addmm(bb, x2, wb.t()) if bb is not None else torch.mm(x2, wb.t())
            if act == "relu":
                y = torch.relu(y)
            elif act == "gelu":
                y = F.gelu(y)
        ctx.save_for_backward(x2, w, y if act == "relu" else None, pre)
        ctx.act, ctx.has_bias, ctx.bias_ref = act, bias is not None, bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y, pre = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        dx = dw = db = None
        bias_done = False
        if ctx.has_bias and ctx.needs_input_grad[2]:
            # one native pass: activation backward + fp32 bias-gradient column sums, accumulated
            # straight into the flat gradient when the engine owns one (csrc/kernels/bn.hip
            # act_bwd_reduce_kernel)
            bias = ctx.bias_ref
            bbuf = grad_slot(bias) if bias is not None else None
            z = y if ctx.act == "relu" else (pre if ctx.act == "gelu" else None)
            outs = native().act_bwd_reduce(dy, z, True, bbuf, ctx.act == "gelu")
            dy = outs[0]
            if bbuf is not None:
                hook = getattr(bias, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(bias)
            else:
                db = outs[1].to(bias.dtype)
            bias_done = True
        elif ctx.act == "relu":
            dy = dy * (y > 0).to(dy.dtype)
        elif ctx.act == "gelu":
            dy = torch.ops.aten.gelu_backward(dy, pre)
        ga = ctx.grad_add
        if ga is not None and ga.grad is not None:
            # residual gradient of x folded into the data-gradient GEMM (beta = 1)
            g = ga.grad.reshape(dy.shape[0], -1).to(torch.bfloat16)
            ga.grad, ga.armed = None, False
            dx = torch.addmm(g, dy, bf16_weight(w)) if ctx.needs_input_grad[0] else g
        elif ctx.needs_input_grad[0]:
            dx = torch.mm(dy, bf16_weight(w))
        if ctx.needs_input_grad[1]:
            gbuf = grad_slot(w)
            if gbuf is not None:
                # accumulate straight into the flat fp32 gradient (bf16 in, fp32 out)
                g2 = gbuf.view(dy.shape[1], x2.shape[1])
                if _use_wgrad256(dy, x2):
                    native().linear_wgrad(dy.contiguous(), x2, g2)
                elif not _blas_accumulate(g2, dy, x2):
                    g2.add_(torch.mm(dy.t(), x2, out_dtype=torch.float32))
                hook = getattr(w, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(w)
            elif _use_wgrad256(dy, x2):
                g2 = torch.zeros(dy.shape[1], x2.shape[1], device=dy.device, dtype=torch.float32)
                native().linear_wgrad(dy.contiguous(), x2, g2)
                dw = g2.to(w.dtype)
            else:
                dw = torch.mm(dy.t(), x2, out_dtype=torch.float32).to(w.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2] and not bias_done:
            bias = ctx.bias_ref
            db = torch.sum(dy, 0, dtype=torch.float32)   # fp32 accumulation, no fp32 copy of dy
            bbuf = grad_slot(bias) if bias is not None else None
            if bbuf is not None:
                bbuf.add_(db)
                hook = getattr(bias, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(bias)
                db = None
        return dx, dw, db, None, None, None


class _LinearNativeFn(torch.autograd.Function):
    """Transformer-size linear on the hand-written MFMA kernels (igemm / igemm2, zoo._C):

      forward   y = act(x W^T + b): GEMM with the bias (+ReLU) epilogue; GELU keeps its bf16
                pre-activation beside the output from the same epilogue (its backward needs it)
      backward  one native pass computes the activation backward and the fp32 bias-gradient
                column sums (straight into the engine's flat gradient); dX = dY W on the GEMM
                with the residual gradient (GradAdd) added in its epilogue; W^T is the cached
                1x1 "flipped" weight (refreshed in the batched flip launch after each update);
                dW += dY^T X on the 256x256 LDS-DMA weight-gradient kernel into the flat grad.
    Reference: TransformerLayer.scala:120-181 / BERT.scala Dense layers."""

    @staticmethod
    def forward(ctx, x2, w, bias, act, need_grad, grad_add=None, gelu_link=None, gelu_src=None):
        ctx.grad_add = grad_add
        if grad_add is not None and need_grad:
            grad_add.armed = True
        N, K = w.shape
        wb = bf16_weight(w)
        bf = None if bias is None else bias.detach().float().contiguous()
        x4 = x2.view(x2.shape[0], 1, 1, K)
        pre = None
        if act == "gelu" and need_grad and not _GELU_DUAL:
            pre = _kern.conv_fwd(x4, wb, 1, 1, bias=bf).view(-1, N)
            y = native().act_fwd_bwd(pre, None, 4, 0.0)
        elif act == "gelu" and need_grad:
            # one GEMM writes both gelu(v) and v (its backward's operand): igemm2.hip EPI 3 stores
            # the pre-activation beside the output, no separate GELU pass over v
            pre4 = torch.empty(x2.shape[0], 1, 1, N, dtype=torch.bfloat16, device=x2.device)
            y = _kern.conv_fwd(x4, wb, 1, 1, bias=bf, act=ACT_CODES[act], act_pre=pre4).view(-1, N)
            pre = pre4.view(-1, N)
        else:
            y = _kern.conv_fwd(x4, wb, 1, 1, bias=bf, act=ACT_CODES[act]).view(-1, N)
        ctx.gelu_link = ctx.gelu_src = None
        if gelu_link is not None and pre is not None:
            gelu_link.pre, gelu_link.y, gelu_link.db, gelu_link.done = pre, y, None, False
            ctx.gelu_link = gelu_link
        if (gelu_src is not None and need_grad and gelu_src.pre is not None and gelu_src.y is not None and
                gelu_src.y.data_ptr() == x2.data_ptr() and gelu_src.y.shape == x2.shape):
            ctx.gelu_src = gelu_src            # x2 IS the GELU output of the linked linear
        ctx.save_for_backward(x2, w, y if act == "relu" else None, pre)
        ctx.act, ctx.has_bias, ctx.bias_ref = act, bias is not None, bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y, pre = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        N, K = w.shape
        dx = dw = db = None
        link = ctx.gelu_link
        if link is not None and link.done:
            # the consuming linear already applied GELU' in its dgrad epilogue (dy = d pre)
            # and summed the bias gradient there
            if ctx.has_bias and ctx.needs_input_grad[2]:
                bias = ctx.bias_ref
                bbuf = grad_slot(bias)
                if bbuf is not None:
                    # a bias-gradient add nothing on the data-gradient path waits for: side stream
                    with wstream.wgrad(dy.device, link.db, on=True):
                        bbuf.add_(link.db)
                        hook = getattr(bias, "_zoo_grad_ready", None)
                        if hook is not None:
                            hook(bias)
                else:
                    db = link.db.to(bias.dtype)
            link.pre = link.y = link.db = None
            link.done = False
        elif (ctx.has_bias and ctx.needs_input_grad[2]) or ctx.act in ("relu", "gelu"):
            bias = ctx.bias_ref
            want_db = bool(ctx.has_bias and ctx.needs_input_grad[2])
            bbuf = grad_slot(bias) if (want_db and bias is not None) else None
            z = y if ctx.act == "relu" else (pre if ctx.act == "gelu" else None)
            # no activation: the pass only sums dy's columns into the engine-owned bias gradient,
            # nothing on the data-gradient path waits for it -> weight-gradient side stream
            with wstream.wgrad(dy.device, dy, on=z is None and bbuf is not None):
                outs = native().act_bwd_reduce(dy, z, want_db, bbuf, ctx.act == "gelu")
                if want_db and bbuf is not None:
                    hook = getattr(bias, "_zoo_grad_ready", None)
                    if hook is not None:
                        hook(bias)
            dy = outs[0]
            if want_db and bbuf is None:
                db = outs[1].to(bias.dtype)
        ga = ctx.grad_add
        resid = None
        if ga is not None and ga.grad is not None:
            resid = ga.grad.reshape(dy.shape[0], K).to(torch.bfloat16).contiguous()
            ga.grad, ga.armed = None, False
        src = ctx.gelu_src
        if ctx.needs_input_grad[0] and src is not None and src.pre is not None:
            # dgrad epilogue: d pre = (dy W^T (+ resid)) * GELU'(pre), column sums -> b1's gradient
            wt = _kern.flip_weights(bf16_weight(w), N, 1, 1, K)
            # per-step arena (zeroed once per engine step) instead of a fill launch per layer
            from zoo.ops import workspace
            sums = workspace.zeros(2 * K, dy.device)
            dx = _kern.conv_fwd(dy.view(-1, 1, 1, N), wt, 1, 1,
                                resid=None if resid is None else resid.view(-1, 1, 1, K),
                                bstats=(src.pre.view(-1, 1, 1, K), None, None, None, sums)).view(-1, K)
            src.db, src.done = sums[:K], True
        elif ctx.needs_input_grad[0]:
            wt = _kern.flip_weights(bf16_weight(w), N, 1, 1, K)       # W^T [K, ceil8(N)]
            dx = _kern.conv_fwd(dy.view(-1, 1, 1, N), wt, 1, 1,
                                resid=None if resid is None else resid.view(-1, 1, 1, K)).view(-1, K)
        elif resid is not None:
            dx = resid
        if ctx.needs_input_grad[1]:
            gbuf = grad_slot(w)
            g2 = gbuf.view(N, K) if gbuf is not None else torch.zeros(N, K, device=dy.device, dtype=torch.float32)
            # engine-owned gradient: on the weight-gradient side stream (zoo.ops.wstream)
            with wstream.wgrad(dy.device, dy, x2, on=gbuf is not None):
                native().linear_wgrad(dy, x2, g2)
                if gbuf is not None:
                    hook = getattr(w, "_zoo_grad_ready", None)
                    if hook is not None:
                        hook(w)
            if gbuf is None:
                dw = g2.to(w.dtype)
        return dx, dw, db, None, None, None, None, None


def _use_native_linear(x, Cin, K, act):
    M = x.numel() // max(Cin, 1)
    return M >= 1024 and Cin >= 256 and K >= 256 and Cin % 8 == 0 and K % 8 == 0 and \
        act in (None, "linear", "relu", "gelu")


_ADDMM_DTYPE_OK = [True]
# GELU backward in the consuming linear's dgrad epilogue (GeluLink); ZOO_GELU_DGRAD=0 restores the
# separate activation-backward pass
_GELU_DGRAD = True
_WGRAD256 = True


def _use_wgrad256(dy, x2):
    """The 256x256-tile LDS-DMA weight-gradient kernel (csrc/kernels/wgrad256.hip) beats
    hipBLASLt's fp32-output GEMM 1.6-2.2x at transformer shapes (tall reduction, small
    weight: tools/wgrad_bench.py); hipBLASLt keeps very large weights (>= 16M elements),
    where the library's main loop is faster and no split of the reduction is needed."""
    N, K = dy.shape[1], x2.shape[1]
    return (_WGRAD256 and dy.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and N % 8 == 0 and
            K % 8 == 0 and N * K < (1 << 24) and N >= 128 and K >= 128 and x2.stride(1) == 1 and
            x2.stride(0) % 8 == 0)


def _blas_accumulate(g2, dy, x2):
    """g2 (fp32) += dy^T x2 (bf16) in one hipBLASLt call; False if unsupported here."""
    if not _ADDMM_DTYPE_OK[0]:
        return False
    try:
        torch.ops.aten.addmm.dtype_out(g2, dy.t(), x2, torch.float32, beta=1, alpha=1, out=g2)
        return True
    except (RuntimeError, TypeError, AttributeError):
        _ADDMM_DTYPE_OK[0] = False
        return False


def _bf16_bias(bias):
    """bf16 copy of a bias vector, cached on the parameter until it changes (an
    inference model converts it once instead of every call)."""
    c = getattr(bias, "_zoo_bf16_bias", None)
    if c is not None and c[0] == bias._version and c[1].data_ptr() != 0 and c[2] == bias.data_ptr():
        return c[1]
    b = bias.detach().to(torch.bfloat16)
    try:
        bias._zoo_bf16_bias = (bias._version, b, bias.data_ptr())
    except (AttributeError, RuntimeError):
        pass
    return b


def _use_blas(x, Cin, K, act):
    M = x.numel() // max(Cin, 1)
    return _BLAS_LINEAR and M >= 1024 and Cin >= 256 and K >= 256 and Cin % 8 == 0 and K % 8 == 0 and \
        act in (None, "linear", "relu", "gelu")


def linear(x, w, bias=None, act=None, grad_add=None, gelu_link=None, gelu_src=None):
    """y = act(x @ w^T + b). Uses the MFMA GEMM when features are 8-aligned and
    the input is on the GPU; otherwise the plain library GEMM (hipBLASLt).
    ``grad_add``: a :class:`zoo.ops.nn.GradAdd` whose residual gradient the data-gradient
    GEMM adds (only armed on the library-GEMM path; elsewhere autograd sums as usual).
    ``gelu_link`` / ``gelu_src``: a :class:`zoo.ops.nn.GeluLink` joining a GELU linear to the
    linear that consumes its output (native path only; ignored elsewhere)."""
    K, Cin = w.shape
    lead = x.shape[:-1]
    if x.is_cuda and (Cin % 8 or K % 8) and x.shape[-1] == Cin:
        # zero-pad features to the MFMA kernels' 8-element granule (keeps small
        # layers such as NCF's 30->10->5 off hipBLASLt's tall-skinny fp32 wgrad)
        pc, pk = (-Cin) % 8, (-K) % 8
        xp = F.pad(x, (0, pc)) if pc else x
        wp = F.pad(w, (0, pc, 0, pk))
        bp = None if bias is None or not pk else F.pad(bias, (0, pk))
        return linear(xp, wp, bias if bp is None else bp, act)[..., :K]
    if x.is_cuda and w.shape[1] == Cin and x.shape[-1] == Cin and _use_blas(x, Cin, K, act):
        xb = x.reshape(-1, Cin)
        xb = (xb if xb.dtype == torch.bfloat16 else xb.to(torch.bfloat16)).contiguous()
        need_grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or
                                                  (bias is not None and bias.requires_grad))
        y = _LinearBlasFn.apply(xb, w, bias, None if act == "linear" else act, need_grad, grad_add)
        return y.reshape(*lead, K).to(x.dtype)
    if x.is_cuda and w.shape[1] == Cin and x.shape[-1] == Cin and _use_native_linear(x, Cin, K, act):
        xb = x.reshape(-1, Cin)
        xb = (xb if xb.dtype == torch.bfloat16 else xb.to(torch.bfloat16)).contiguous()
        need_grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or
                                                  (bias is not None and bias.requires_grad))
        y = _LinearNativeFn.apply(xb, w, bias, None if act == "linear" else act, need_grad, grad_add,
                                  gelu_link if _GELU_DGRAD else None, gelu_src if _GELU_DGRAD else None)
        return y.reshape(*lead, K).to(x.dtype)
    if x.is_cuda and Cin % 8 == 0 and K % 8 == 0 and w.shape[1] == Cin:
        x2 = x.reshape(-1, 1, 1, Cin)
        out_f32 = x.dtype == torch.float32
        y = conv2d_nhwc(x2, w, bias, act=act, out_f32=out_f32)
        return y.reshape(*lead, K).to(x.dtype)
    y = F.linear(x, w.to(x.dtype), None if bias is None else bias.to(x.dtype))
    return _ref_act(y, act)


class _ConvTranspose2dFn(torch.autograd.Function):
    """Transposed conv (Deconvolution2D) = data-gradient of the conv F whose
    packed weight is ``wf`` [Cin_deconv, R*S*Cout_deconv]. Forward runs the
    dgrad kernel path (input dilation = stride); backward is a plain forward
    conv (dX) and a wgrad with the operands' roles swapped (dW)."""

    @staticmethod
    def forward(ctx, x, wf, R, S, stride, pad, out_hw, cout):
        cin = x.shape[3]
        y = _kern.conv_dgrad(x, bf16_weight(wf), cin, R, S, cout, out_hw[0], out_hw[1], stride, pad)
        ctx.save_for_backward(x, wf)
        ctx.g = (R, S, stride, pad, cout)
        return y

    @staticmethod
    def backward(ctx, dy):
        C_ = native()
        x, wf = ctx.saved_tensors
        R, S, stride, pad, cout = ctx.g
        dyb = dy.contiguous().to(torch.bfloat16)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _kern.conv_fwd(dyb, bf16_weight(wf), R, S, stride, pad, out_hw=(x.shape[1], x.shape[2]))
        if ctx.needs_input_grad[1]:
            gw = torch.zeros(wf.shape, dtype=torch.float32, device=wf.device)
            C_.conv_wgrad(dyb, x, gw, R, S, stride[0], stride[1], pad[0], pad[1], 1, 1)
            dw = gw.to(wf.dtype)
        return dx, dw, None, None, None, None, None, None


def conv_transpose2d_nhwc(x, wf, kernel, stride, pad, out_hw, cout):
    """x: [N,H,W,Cin]; wf: packed [Cin, ceil8(R*S*Cout)] (Wf[ci][r][s][co] = Wd[ci][co][r][s])."""
    R, S = kernel
    if x.is_cuda:
        return _ConvTranspose2dFn.apply(x.to(torch.bfloat16).contiguous(), wf, R, S, tuple(stride), tuple(pad),
                                        tuple(out_hw), cout)
    cin = x.shape[3]
    wd = unpack_weight(wf.float(), cin, R, S, cout).permute(0, 3, 1, 2)  # [ci][co][r][s]
    H, W = x.shape[1], x.shape[2]
    oh = (H - 1) * stride[0] - 2 * pad[0] + R
    ow = (W - 1) * stride[1] - 2 * pad[1] + S
    y = F.conv_transpose2d(x.float().permute(0, 3, 1, 2), wd, stride=stride, padding=pad,
                           output_padding=(out_hw[0] - oh, out_hw[1] - ow))
    return y.permute(0, 2, 3, 1).to(x.dtype)
