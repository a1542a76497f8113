"""TransformerLayer (GPT-style, optional causal mask) and BERT.

Parity: Py/pipeline/api/keras/layers/self_attention.py,
Zs/pipeline/api/keras/layers/TransformerLayer.scala:56-279 (block 120-127,
mlp 129-135, multiHeadSelfAttention 137-161, attn 163-181) and BERT.scala:66-402
(defaults: vocab 40990, hidden 768, 12 blocks, 12 heads, max position 512,
intermediate 3072; GELU via erf 88-92; additive mask (1-mask)*-10000 94-105).

Built directly from native ops: fused QKV projection (one MFMA GEMM),
attention (``zoo.ops.attention``), LayerNorm (native row kernel), GELU.
Inputs/outputs follow the reference:
  TransformerLayer: [token_ids, position_ids] -> [sequence_output, pooled]
  BERT: [token_ids, token_type_ids, position_ids, attention_mask]
        -> [block outputs..., pooled] (all blocks) or [last, pooled]
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.ops.attention import attention_packed
from zoo.ops.nn import GeluLink, GradAdd, dropout_add, dropout_add_layer_norm
from zoo.ops.pointwise import dropout as ops_dropout
from zoo.pipeline.api.keras.base import Layer


# residual-gradient handoff into the linear's dgrad GEMM (GradAdd): measured neutral on
# BERT-base b128 (same-box A/B 17.13/17.15 ms off vs 17.24/17.15 on: hipBLASLt's beta=1
# epilogue costs what the separate add did), so opt-in
_RESID_GRAD_FUSE = False
# residual gradient summed inside the producing LayerNorm's backward kernel instead (the
# LayerNorm that made x / n is armed; the residual dropout_add parks its gradient there)
_LN_GRAD_ADD = True
# residual dropout-add fused into the LayerNorm forward (one pass: the sum is stored for the
# backward but never read back), ops.nn.dropout_add_layer_norm
_DROP_LN_FUSE = True


def _res_ln(a, x, p, training, gamma, beta, eps, grad_add, grad_in):
    if _DROP_LN_FUSE:
        return dropout_add_layer_norm(a, x, p, training, gamma, beta, eps, grad_add=grad_add, grad_in=grad_in)
    return ops.layer_norm(dropout_add(a, x, p, training, grad_add=grad_add), gamma, beta, eps, grad_in=grad_in)


def _normal(shape, std):
    t = torch.empty(shape)
    nn.init.normal_(t, 0.0, std)
    return t


class _Block(nn.Module):
    def __init__(self, hidden, n_head, inter, hidden_drop, attn_drop, init_range, post_ln=True, gelu="erf",
                 ln_eps=1e-5):
        super().__init__()
        self.ln_eps = float(ln_eps)
        self.h, self.n_head = hidden, n_head
        self.qkv_w = nn.Parameter(_normal((3 * hidden, hidden), init_range))
        self.qkv_b = nn.Parameter(torch.zeros(3 * hidden))
        self.proj_w = nn.Parameter(_normal((hidden, hidden), init_range))
        self.proj_b = nn.Parameter(torch.zeros(hidden))
        self.ln1_g, self.ln1_b = nn.Parameter(torch.ones(hidden)), nn.Parameter(torch.zeros(hidden))
        self.fc1_w = nn.Parameter(_normal((inter, hidden), init_range))
        self.fc1_b = nn.Parameter(torch.zeros(inter))
        self.fc2_w = nn.Parameter(_normal((hidden, inter), init_range))
        self.fc2_b = nn.Parameter(torch.zeros(hidden))
        self.ln2_g, self.ln2_b = nn.Parameter(torch.ones(hidden)), nn.Parameter(torch.zeros(hidden))
        self.hidden_drop, self.attn_drop, self.gelu = hidden_drop, attn_drop, gelu

    def forward(self, x, mask=None, causal=False):
        B, L, H = x.shape
        nh, hd = self.n_head, H // self.n_head
        # x and n each feed a linear and a residual add: the add's x-gradient is folded into
        # the linear's data-gradient GEMM (GradAdd) instead of a separate autograd sum
        h1, h2 = (GradAdd(), GradAdd()) if _RESID_GRAD_FUSE else (None, None)
        # ... or into the backward of the LayerNorm that produced x (the previous block's output
        # LayerNorm, which attached its holder to x) and n (this block's first LayerNorm)
        lx = ln_n = ln_out = None
        if h1 is None and _LN_GRAD_ADD and x.is_cuda and torch.is_grad_enabled():
            lx = getattr(x, "_zoo_grad_in", None)
            ln_n, ln_out = GradAdd(), GradAdd()
        qkv = ops.linear(x, self.qkv_w, self.qkv_b, grad_add=h1)     # [B, L, 3H]
        # strided fused kernels (attention-probability dropout in-kernel), no head copies
        a = attention_packed(qkv, nh, mask=mask, causal=causal, dropout_p=self.attn_drop, training=self.training)
        if a is None:
            qkv = qkv.reshape(B, L, 3, nh, hd).permute(2, 0, 3, 1, 4)  # [3, B, nh, L, hd]
            a = ops.attention(qkv[0], qkv[1], qkv[2], mask=mask, causal=causal, dropout_p=self.attn_drop,
                              training=self.training)
            a = a.transpose(1, 2).reshape(B, L, H)
        a = ops.linear(a, self.proj_w, self.proj_b)
        n = _res_ln(a, x, self.hidden_drop, self.training, self.ln1_g, self.ln1_b, self.ln_eps,
                    h1 if h1 is not None else lx, ln_n)
        act = "gelu" if self.gelu == "erf" else None
        gl = GeluLink() if act == "gelu" else None      # GELU backward in fc2's dgrad epilogue
        m = ops.linear(n, self.fc1_w, self.fc1_b, act=act, grad_add=h2, gelu_link=gl)
        if self.gelu != "erf":  # GPT tanh approximation
            m = 0.5 * m * (1 + torch.tanh(math.sqrt(2 / math.pi) * (m + 0.044715 * m * m * m)))
        m = ops.linear(m, self.fc2_w, self.fc2_b, gelu_src=gl)
        out = _res_ln(m, n, self.hidden_drop, self.training, self.ln2_g, self.ln2_b, self.ln_eps,
                      h2 if h2 is not None else ln_n, ln_out)
        if ln_out is not None:
            out._zoo_grad_in = ln_out   # the next block's residual parks its x-gradient here
        return out


class TransformerLayer(Layer):
    def __init__(self, n_block, hidden_drop, attn_drop, n_head, initializer_range, bidirectional,
                 output_all_block, embedding_layer=None, input_shape=None, intermediate_size=0, vocab=40990,
                 hidden_size=768, embedding_drop=0.1, **kwargs):
        super().__init__(input_shape=None, **kwargs)
        self._given_input_shape = input_shape
        self.n_block, self.n_head, self.bidirectional = n_block, n_head, bidirectional
        self.output_all_block = output_all_block
        self.seq_len = input_shape[0][0] if input_shape else None
        self.hidden = hidden_size
        self.embedding_layer = embedding_layer
        if embedding_layer is None:
            self.tok = nn.Parameter(_normal((vocab, hidden_size), initializer_range))
            self.embedding_drop = embedding_drop
        inter = intermediate_size if intermediate_size > 0 else 4 * hidden_size
        self.blocks = nn.ModuleList([_Block(hidden_size, n_head, inter, hidden_drop, attn_drop, initializer_range,
                                            gelu="tanh") for _ in range(n_block)])
        self.pool_w = nn.Parameter(_normal((hidden_size, hidden_size), initializer_range))
        self.pool_b = nn.Parameter(torch.zeros(hidden_size))
        self.built = True

    @classmethod
    def init(cls, vocab=40990, seq_len=77, n_block=12, hidden_drop=0.1, attn_drop=0.1, n_head=12, hidden_size=768,
             embedding_drop=0.1, initializer_range=0.02, bidirectional=False, output_all_block=False):
        return cls(n_block, hidden_drop, attn_drop, n_head, initializer_range, bidirectional, output_all_block,
                   None, ((seq_len,), (seq_len,)), 0, vocab, hidden_size, embedding_drop)

    def compute_output_shape(self, input_shape):
        L = input_shape[0][1]
        seq = (None, L, self.hidden)
        if self.output_all_block:
            return [seq] * self.n_block + [(None, self.hidden)]
        return [seq, (None, self.hidden)]

    def _embed(self, xs):
        tok, pos = xs[0].long(), xs[1].long()
        if self.embedding_layer is not None:
            return self.embedding_layer([xs[0], xs[1]])
        # reference: one table shared by word and position ids, summed
        e = ops.embedding(tok, self.tok) + ops.embedding(pos, self.tok)
        if e.is_cuda:
            e = e.to(torch.bfloat16)
        return ops_dropout(e, self.embedding_drop, self.training)

    def call(self, xs):
        x = self._embed(xs)
        outs = []
        for blk in self.blocks:
            x = blk(x, None, causal=not self.bidirectional)
            outs.append(x)
        pooled = torch.tanh(ops.linear(x[:, 0], self.pool_w, self.pool_b))
        return outs + [pooled] if self.output_all_block else [x, pooled]


class BERT(Layer):
    def __init__(self, vocab=40990, hidden_size=768, n_block=12, n_head=12, max_position_len=512,
                 intermediate_size=3072, hidden_drop=0.1, attn_drop=0.1, initializer_range=0.02,
                 output_all_block=True, input_shape=None, seq_len=None, type_vocab_size=2, layer_norm_eps=1e-5,
                 **kwargs):
        super().__init__(input_shape=None, **kwargs)
        self.vocab, self.hidden, self.n_block, self.n_head = vocab, hidden_size, n_block, n_head
        self.max_position_len, self.output_all_block = max_position_len, output_all_block
        self.seq_len = seq_len
        self.word = nn.Parameter(_normal((vocab, hidden_size), initializer_range))
        self.position = nn.Parameter(_normal((max_position_len, hidden_size), initializer_range))
        self.token_type = nn.Parameter(_normal((type_vocab_size, hidden_size), initializer_range))
        self.layer_norm_eps = float(layer_norm_eps)
        self.emb_ln_g, self.emb_ln_b = nn.Parameter(torch.ones(hidden_size)), nn.Parameter(torch.zeros(hidden_size))
        self.hidden_drop = hidden_drop
        self.blocks = nn.ModuleList([_Block(hidden_size, n_head, intermediate_size, hidden_drop, attn_drop,
                                            initializer_range, gelu="erf", ln_eps=layer_norm_eps)
                                     for _ in range(n_block)])
        self.pool_w = nn.Parameter(_normal((hidden_size, hidden_size), initializer_range))
        self.pool_b = nn.Parameter(torch.zeros(hidden_size))
        self.built = True

    @classmethod
    def init(cls, vocab=40990, hidden_size=768, n_block=12, n_head=12, seq_len=512, intermediate_size=3072,
             hidden_drop=0.1, attn_drop=0.1, initializer_range=0.02, output_all_block=True):
        return cls(vocab, hidden_size, n_block, n_head, seq_len, intermediate_size, hidden_drop, attn_drop,
                   initializer_range, output_all_block, seq_len=seq_len)

    def compute_output_shape(self, input_shape):
        L = input_shape[0][1]
        seq = (None, L, self.hidden)
        if self.output_all_block:
            return [seq] * self.n_block + [(None, self.hidden)]
        return [seq, (None, self.hidden)]

    def call(self, xs):
        tok, typ, pos = xs[0].long(), xs[1].long(), xs[2].long()
        amask = xs[3] if len(xs) > 3 else None
        e = ops.embedding(tok, self.word) + ops.embedding(typ, self.token_type) + ops.embedding(pos, self.position)
        if e.is_cuda:  # bf16 activations end to end on the GPU (LayerNorm / attention / GEMMs all take bf16)
            e = e.to(torch.bfloat16)
        x = ops_dropout(ops.layer_norm(e, self.emb_ln_g, self.emb_ln_b, self.layer_norm_eps), self.hidden_drop,
                        self.training)
        mask = None
        if amask is not None:
            mask = (1.0 - amask.float()) * -10000.0  # [B, L] additive key mask (BERT.scala:94-105)
        outs = []
        for blk in self.blocks:
            x = blk(x, mask, causal=False)
            outs.append(x)
        pooled = torch.tanh(ops.linear(x[:, 0], self.pool_w, self.pool_b))
        return outs + [pooled] if self.output_all_block else [x, pooled]
