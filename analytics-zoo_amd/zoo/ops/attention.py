"""Scaled dot-product attention (TransformerLayer.attn, TransformerLayer.scala:163-181).

``attention(q, k, v, mask=None, causal=False, dropout_p=0.0)`` with q/k/v
shaped [batch, heads, seq, head_dim]. On the GPU with head_dim in {64, 128},
no dropout and a causal and/or additive [B, S] key mask, the fused native HIP
kernel runs (csrc/kernels/attention.hip: online softmax, O(L) memory, bf16
MFMA; ``zoo._C.attn_fwd``/``attn_bwd``). Other configurations (dropout on the
probabilities, general masks) take the materialised path (two batched GEMMs
around a softmax), which is also the CPU implementation.
"""
import math

import torch

from zoo.ops._native import available, native


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
    def forward(ctx, q, k, v, mask, causal):
        o, lse = native().attn_fwd(q, k, v, mask, causal)
        ctx.save_for_backward(q, k, v, mask, o, lse)
        ctx.causal = causal
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, mask, o, lse = ctx.saved_tensors
        dq, dk, dv = native().attn_bwd(do.to(torch.bfloat16).contiguous(), q, k, v, mask, o, lse, ctx.causal)
        return dq, dk, dv, None, None


def _native_ok(q, k, v, mask, dropout_p, training):
    if not q.is_cuda:
        return False
    if q.shape[-1] not in (64, 128) or (dropout_p > 0 and training) or q.dim() != 4:
        return False
    if mask is not None and (mask.dim() != 2 or tuple(mask.shape) != (q.shape[0], k.shape[-2])):
        return False
    if not available():
        raise RuntimeError("zoo native kernels are not built: run tools/build_native.py (fused attention)")
    return True


def attention_packed(qkv, n_head, mask=None, causal=False):
    """Inference attention straight from a packed [B, L, 3*H*D] QKV projection:
    the fused kernel reads q/k/v through strides and writes [B, L, H*D], so the
    per-head permute copies disappear. Returns None when the fused kernel does
    not apply (caller falls back to :func:`attention`)."""
    B, L, three_h = qkv.shape
    hd = three_h // (3 * n_head)
    if not (qkv.is_cuda and qkv.dtype == torch.bfloat16 and hd in (64, 128) and qkv.is_contiguous()):
        return None
    if torch.is_grad_enabled() and qkv.requires_grad:
        return None
    if mask is not None and (mask.dim() != 2 or tuple(mask.shape) != (B, L)):
        return None
    v5 = qkv.view(B, L, 3, n_head, hd).permute(2, 0, 3, 1, 4)   # [3, B, H, L, hd] strided views
    o, _ = native().attn_fwd_strided(v5[0], v5[1], v5[2], None if mask is None else mask.float().contiguous(),
                                     bool(causal), True)
    return o.view(B, L, n_head * hd)


def attention(q, k, v, mask=None, causal=False, dropout_p=0.0, training=False):
    """mask: additive float mask broadcastable to [B, H, L, S]; a [B, S] key
    mask (0 keep / -10000 drop, BERT style) takes the fused path."""
    if _native_ok(q, k, v, mask, dropout_p, training):
        dt = q.dtype
        bf = torch.bfloat16
        o = _FlashAttnFn.apply(q.to(bf).contiguous(), k.to(bf).contiguous(), v.to(bf).contiguous(),
                               None if mask is None else mask.float().contiguous(), bool(causal))
        return o if dt == bf else o.to(dt)
    m = mask
    if m is not None and m.dim() == 2:
        m = m[:, None, None, :]
    return _reference(q, k, v, m, causal, dropout_p, training)
