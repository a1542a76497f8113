"""Fused softmax + cross-entropy (ClassNLL over log-softmax) on gfx950.

Forward and backward are computed by ONE kernel launch: the gradient w.r.t.
the logits, ``(softmax - onehot) * scale``, is produced in the forward pass and
returned from backward (scaled by the incoming grad), so the loss costs one
read of the logits. Honours the padding label of ZooClassNLLCriterion
(Zs/pipeline/api/keras/objectives/ZooClassNLLCriterion.scala:28-100).
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native


class _SoftmaxXentAtomicFn(torch.autograd.Function):
    """The round-5 formulation (atomic sums, clamp / div / mul / cast launches): A/B oracle."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        outs = native().softmax_xent(logits, labels, True, 1.0, ignore_index)
        acc, dl = outs[0], outs[1]
        count = acc[1].clamp_min(1.0)
        ctx.save_for_backward(dl, count)
        return acc[0] / count

    @staticmethod
    def backward(ctx, g):
        dl, count = ctx.saved_tensors
        return dl * (g / count).to(dl.dtype), None, None


_XENT_MEAN = True   # A/B switch: False = _SoftmaxXentAtomicFn


class _SoftmaxXentFn(torch.autograd.Function):
    """Two launches forward (per-row terms + the ordered fold into [mean, count]: deterministic,
    no accumulator fill / clamp / div launches), one backward (dlogits * g / count in the logits
    dtype)."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        out, dl = native().softmax_xent_mean(logits, labels, ignore_index)
        ctx.save_for_backward(dl, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        dl, out = ctx.saved_tensors
        return native().xent_grad_scale(dl, g.float().reshape(1).contiguous(), out[1:2]), None, None


def softmax_cross_entropy(logits, labels, ignore_index=-100):
    """Mean cross-entropy of raw logits [B, C] against int64 labels [B]."""
    labels = labels.long()
    if logits.is_cuda and logits.dtype in (torch.float32, torch.bfloat16) and logits.shape[0] > 0:
        fn = _SoftmaxXentFn if _XENT_MEAN else _SoftmaxXentAtomicFn
        return fn.apply(logits.contiguous(), labels.contiguous(), int(ignore_index))
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index)


class _ProbNllFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, probs, labels, eps, ignore_index, size_average):
        # [loss, count] from the native pass + its ordered fold (no accumulator fill, no clamp /
        # div launches); the backward scales by 1 / max(count, 1) itself
        out = native().prob_nll_mean(probs, labels, eps, ignore_index, size_average)
        ctx.save_for_backward(probs, labels, out[1:2])
        ctx.eps, ctx.ignore, ctx.avg = eps, ignore_index, size_average
        return out[0]

    @staticmethod
    def backward(ctx, g):
        probs, labels, count = ctx.saved_tensors
        if not ctx.avg:
            count = torch.ones_like(count)
        dp = native().prob_nll_grad(probs, labels, g.float().reshape(1).contiguous(), count, ctx.eps, ctx.ignore)
        return dp.to(probs.dtype), None, None, None, None


def prob_nll(probs, labels, eps=1e-7, ignore_index=-100, size_average=True):
    """-mean(log(clamp(probs[i, label_i], eps, 1))) over non-ignored rows (ClassNLLCriterion on
    probabilities): one native pass computes the loss and the (unscaled) gradient."""
    labels = labels.long().reshape(-1)
    if probs.is_cuda and probs.dim() == 2 and probs.dtype in (torch.float32, torch.bfloat16):
        return _ProbNllFn.apply(probs.contiguous(), labels.contiguous(), float(eps), int(ignore_index),
                                bool(size_average))
    logp = torch.log(torch.clamp(probs.float(), eps, 1.0))
    return F.nll_loss(logp, labels, ignore_index=ignore_index, reduction="mean" if size_average else "sum")
