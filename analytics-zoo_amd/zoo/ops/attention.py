"""Scaled dot-product attention (TransformerLayer.attn, TransformerLayer.scala:163-181).

``attention(q, k, v, mask=None, causal=False, dropout_p=0.0)`` with q/k/v
shaped [batch, heads, seq, head_dim]. On the GPU with head_dim in {64, 128}
and a causal and/or additive [B, S] key mask, the fused native HIP kernel runs
(csrc/kernels/attention.hip: online softmax, O(L) memory, bf16 MFMA;
``zoo._C.attn_fwd``/``attn_bwd``). Dropout on the attention probabilities
(BERT's attention_probs dropout) is applied inside the kernel with a counter
hash of (batch*head, query, key, seed), so the backward pass regenerates the
mask instead of storing an [L, S] tensor. General masks take the materialised
path (two batched GEMMs around a softmax), which is also the CPU implementation.
"""
import math

import torch

from zoo.ops._native import available, native
from zoo.ops.pointwise import _seed


def _dropout_seed(device, pdrop):
    """A per-call dropout seed. Under hipGraph capture the kernels XOR in the device seed
    offset (attention.hip), so the capture must record that the graph reads it: the engine
    restages the offset before a replay only when some captured kernel does
    (devscalar.seed_offset_used)."""
    if pdrop <= 0:
        return 0
    if torch.cuda.is_current_stream_capturing():
        from zoo.ops.devscalar import seed_offset_live
        seed_offset_live(device)
    return _seed()


def _reference(q, k, v, mask, causal, dropout_p, training):
    scale = 1.0 / math.sqrt(q.shape[-1])
    w = torch.matmul(q, k.transpose(-1, -2)) * scale
    if causal:
        L, S = w.shape[-2], w.shape[-1]
        tri = torch.ones(L, S, dtype=torch.bool, device=w.device).tril(S - L)
        w = w.masked_fill(~tri, float("-inf"))
    if mask is not None:
        w = w + mask.to(w.dtype)
    p = torch.softmax(w.float(), dim=-1).to(q.dtype)
    if dropout_p > 0 and training:
        p = torch.nn.functional.dropout(p, dropout_p)
    return torch.matmul(p, v)


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, mask, causal, pdrop):
        seed = _dropout_seed(q.device, pdrop)
        o, lse = native().attn_fwd(q, k, v, mask, causal, pdrop, seed)
        ctx.save_for_backward(q, k, v, mask, o, lse)
        ctx.causal, ctx.pdrop, ctx.seed = causal, pdrop, seed
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, mask, o, lse = ctx.saved_tensors
        dq, dk, dv = native().attn_bwd(do.to(torch.bfloat16).contiguous(), q, k, v, mask, o, lse, ctx.causal,
                                       ctx.pdrop, ctx.seed)
        return dq, dk, dv, None, None, None


def _native_ok(q, k, v, mask, dropout_p, training):
    if not q.is_cuda:
        return False
    if q.shape[-1] not in (64, 128) or q.dim() != 4 or (training and dropout_p >= 1.0):
        return False
    if mask is not None and (mask.dim() != 2 or tuple(mask.shape) != (q.shape[0], k.shape[-2])):
        return False
    if not available():
        raise RuntimeError("zoo native kernels are not built: run tools/build_native.py (fused attention)")
    return True


class _FlashAttnPackedFn(torch.autograd.Function):
    """Training attention on a packed [B, L, 3*H*D] projection: forward and backward read
    q/k/v (and dO / O) through strides and write dq/dk/dv straight into the packed
    gradient, so no per-head permute copies are made in either direction."""

    @staticmethod
    def forward(ctx, qkv, mask, causal, pdrop, n_head):
        B, L, three_h = qkv.shape
        hd = three_h // (3 * n_head)
        seed = _dropout_seed(qkv.device, pdrop)
        v5 = qkv.view(B, L, 3, n_head, hd).permute(2, 0, 3, 1, 4)   # [3, B, H, L, hd] strided views
        o, lse = native().attn_fwd_strided(v5[0], v5[1], v5[2], mask, causal, True, pdrop, seed)
        ctx.save_for_backward(qkv, mask, o, lse)
        ctx.causal, ctx.pdrop, ctx.seed, ctx.n_head = causal, pdrop, seed, n_head
        return o.view(B, L, n_head * hd)

    @staticmethod
    def backward(ctx, do):
        qkv, mask, o, lse = ctx.saved_tensors
        B, L, three_h = qkv.shape
        nh = ctx.n_head
        hd = three_h // (3 * nh)
        do4 = do.to(torch.bfloat16).contiguous().view(B, L, nh, hd).transpose(1, 2)
        v5 = qkv.view(B, L, 3, nh, hd).permute(2, 0, 3, 1, 4)
        dqkv = torch.empty_like(qkv)
        d5 = dqkv.view(B, L, 3, nh, hd).permute(2, 0, 3, 1, 4)
        native().attn_bwd_strided(do4, v5[0], v5[1], v5[2], mask, o.transpose(1, 2), lse, d5[0], d5[1], d5[2],
                                  ctx.causal, ctx.pdrop, ctx.seed)
        return dqkv, None, None, None, None


def attention_packed(qkv, n_head, mask=None, causal=False, dropout_p=0.0, training=False):
    """Attention straight from a packed [B, L, 3*H*D] QKV projection: the fused kernels
    read q/k/v through strides and write [B, L, H*D] (and, under autograd, the packed
    [B, L, 3*H*D] gradient), so the per-head permute copies disappear. Returns None
    when the fused kernel does not apply (caller falls back to :func:`attention`)."""
    B, L, three_h = qkv.shape
    hd = three_h // (3 * n_head)
    if not (qkv.is_cuda and qkv.dtype == torch.bfloat16 and hd in (64, 128) and qkv.is_contiguous()):
        return None
    if mask is not None and (mask.dim() != 2 or tuple(mask.shape) != (B, L)):
        return None
    pdrop = float(dropout_p) if training else 0.0
    if pdrop >= 1.0 or not available():
        return None
    m = None if mask is None else mask.float().contiguous()
    if torch.is_grad_enabled() and qkv.requires_grad:
        return _FlashAttnPackedFn.apply(qkv, m, bool(causal), pdrop, n_head)
    v5 = qkv.view(B, L, 3, n_head, hd).permute(2, 0, 3, 1, 4)   # [3, B, H, L, hd] strided views
    o, _ = native().attn_fwd_strided(v5[0], v5[1], v5[2], m, bool(causal), True, pdrop,
                                     _dropout_seed(qkv.device, pdrop))
    return o.view(B, L, n_head * hd)


def attention(q, k, v, mask=None, causal=False, dropout_p=0.0, training=False):
    """mask: additive float mask broadcastable to [B, H, L, S]; a [B, S] key
    mask (0 keep / -10000 drop, BERT style) takes the fused path."""
    if _native_ok(q, k, v, mask, dropout_p, training):
        dt = q.dtype
        bf = torch.bfloat16
        o = _FlashAttnFn.apply(q.to(bf).contiguous(), k.to(bf).contiguous(), v.to(bf).contiguous(),
                               None if mask is None else mask.float().contiguous(), bool(causal),
                               float(dropout_p) if training else 0.0)
        return o if dt == bf else o.to(dt)
    m = mask
    if m is not None and m.dim() == 2:
        m = m[:, None, None, :]
    return _reference(q, k, v, m, causal, dropout_p, training)
