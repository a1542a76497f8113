"""Native pointwise ops for the Keras layers / objectives / metrics (csrc/kernels/pointwise.hip):
activations (HK13), dropout (HK16), elementwise objectives with the gradient produced in the
forward pass (HK20), the threshold-histogram AUC (HK14) and SSD box decoding (HK21).

Each function takes the native path for fp32 / bf16 CUDA tensors and the plain PyTorch
definition otherwise (which is also the numerics oracle of tests/test_gpu_pointwise.py).
"""
import random

import torch
import torch.nn.functional as F

from zoo.ops._native import native

ACT_CODES = {"relu": 0, "relu6": 1, "elu": 2, "selu": 3, "gelu": 4, "gelu_tanh": 5, "sigmoid": 6,
             "hard_sigmoid": 7, "tanh": 8, "softplus": 9, "softsign": 10, "swish": 11, "silu": 11,
             "log_sigmoid": 12, "tanh_shrink": 13, "exponential": 14, "leaky_relu": 15}


def act_ref(x, name, alpha=1.0):
    n = name.lower()
    return {"relu": torch.relu, "relu6": F.relu6, "elu": lambda t: F.elu(t, alpha), "selu": F.selu,
            "gelu": F.gelu, "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"), "sigmoid": torch.sigmoid,
            "hard_sigmoid": lambda t: torch.clamp(0.2 * t + 0.5, 0.0, 1.0), "tanh": torch.tanh,
            "softplus": F.softplus, "softsign": F.softsign, "swish": F.silu, "silu": F.silu,
            "log_sigmoid": F.logsigmoid, "tanh_shrink": F.tanhshrink, "exponential": torch.exp,
            "leaky_relu": lambda t: F.leaky_relu(t, alpha)}[n](x)


def _native_ok(x):
    return x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, code, alpha):
        ctx.save_for_backward(x)
        ctx.code, ctx.alpha = code, alpha
        return native().act_fwd_bwd(x, None, code, alpha)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return native().act_fwd_bwd(x, dy.contiguous().to(x.dtype), ctx.code, ctx.alpha), None, None


def activation(x, name, alpha=None):
    n = name.lower()
    if alpha is None:
        alpha = 0.01 if n == "leaky_relu" else 1.0
    if n in ACT_CODES and _native_ok(x):
        return _ActFn.apply(x.contiguous(), ACT_CODES[n], float(alpha))
    return act_ref(x, n, alpha)


_RNG = []


def _seed():
    if not _RNG:
        _RNG.append(random.Random(torch.initial_seed() ^ 0x5DEECE66D))
    return _RNG[0].getrandbits(62)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        ctx.p, ctx.seed = p, _seed()
        return native().dropout_fwd(x, p, ctx.seed)

    @staticmethod
    def backward(ctx, g):
        # the same counter-hash mask, regenerated (nothing was stored)
        return native().dropout_fwd(g.contiguous(), ctx.p, ctx.seed), None


def dropout(x, p, training=True):
    if not training or p <= 0:
        return x
    # under hipGraph capture the host seed is baked into the graph: native only when the engine
    # registered the per-step device seed offset the kernel xors in (zoo.ops.devscalar)
    if _native_ok(x) and (not torch.cuda.is_current_stream_capturing() or _seed_offset_live(x.device)):
        return _DropoutFn.apply(x.contiguous(), float(p))
    return F.dropout(x, p, True)


def _seed_offset_live(dev):
    from zoo.ops.devscalar import seed_offset_live
    return seed_offset_live(dev)


LOSS_CODES = {"mse": 0, "mae": 1, "smooth_l1": 2, "bce": 3, "bce_logits": 4, "hinge": 5, "squared_hinge": 6,
              "poisson": 7, "mape": 8, "msle": 9, "kld": 10}


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, code, beta, w):
        loss, grad = native().loss_fwd(pred, target, code, beta, w, True)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, go):
        (grad,) = ctx.saved_tensors
        return grad * go.to(grad.dtype), None, None, None, None


def elementwise_loss(pred, target, kind, weight, beta=1.0):
    """sum_i weight * l(pred_i, target_i) on the native kernel (loss and gradient in one pass);
    ``weight`` = 1/N gives the mean. None when the native path does not apply."""
    if not _native_ok(pred) or not torch.is_tensor(target) or target.shape != pred.shape:
        return None
    target = target.to(device=pred.device, dtype=pred.dtype).contiguous()
    return _LossFn.apply(pred.contiguous(), target, LOSS_CODES[kind], float(beta), float(weight))


def auc(scores, labels, nbins=200, lo=0.0, hi=1.0):
    """Area under the ROC curve over ``nbins`` equal score thresholds (the reference AUC
    metric's threshold counting, AUC.scala:128-211); one native histogram pass on the GPU."""
    s = scores.reshape(-1).float().contiguous()
    l = labels.reshape(-1).float().contiguous()
    if s.is_cuda:
        h = native().auc_hist(s, l, int(nbins), float(lo), float(hi)).double()
    else:
        b = ((s - lo) * (nbins / max(hi - lo, 1e-30))).long().clamp_(0, nbins - 1)
        h = torch.zeros(2, nbins, dtype=torch.float64)
        h[0].index_add_(0, b[l > 0.5], torch.ones(int((l > 0.5).sum()), dtype=torch.float64))
        h[1].index_add_(0, b[l <= 0.5], torch.ones(int((l <= 0.5).sum()), dtype=torch.float64))
    pos, neg = h[0], h[1]
    P, N = float(pos.sum()), float(neg.sum())
    if P == 0 or N == 0:
        return 0.0
    # thresholds from high to low: TPR/FPR after admitting each bin (ties within a bin: trapezoid)
    tp = torch.cat([torch.zeros(1, dtype=h.dtype, device=h.device), pos.flip(0).cumsum(0)]) / P
    fp = torch.cat([torch.zeros(1, dtype=h.dtype, device=h.device), neg.flip(0).cumsum(0)]) / N
    return float(((fp[1:] - fp[:-1]) * (tp[1:] + tp[:-1]) * 0.5).sum())


def box_decode(loc, priors, variances=(0.1, 0.2), clip=False):
    """SSD center-size decoding: loc [N, P, 4] offsets + priors [P, 4] (cx, cy, w, h) ->
    corner boxes [N, P, 4]."""
    if loc.is_cuda:
        return native().box_decode(loc.float().contiguous(), priors.float().contiguous().to(loc.device),
                                   float(variances[0]), float(variances[1]), bool(clip))
    p = priors.to(loc.device).float()
    c = p[None, :, :2] + loc[..., :2] * variances[0] * p[None, :, 2:]
    wh = p[None, :, 2:] * torch.exp(loc[..., 2:] * variances[1])
    b = torch.cat([c - wh / 2, c + wh / 2], -1)
    return b.clamp(0, 1) if clip else b
