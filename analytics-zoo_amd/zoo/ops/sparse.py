"""Embedding-bag and sparse-linear ops on the native
``sparse.hip`` kernels.

* :func:`embedding_bag` -- BigDL ``LookupTableSparse`` semantics
  (``Zs/pipeline/api/keras/layers/SparseEmbedding.scala:76-88``): per-bag
  combination of the looked-up rows, ``combiner`` in {sum, mean, sqrtn} with
  optional per-id weights (the values of a sparse input) and ``max_norm`` row
  renormalisation. Bags are given either as a dense padded id matrix [B, L]
  (ids < 0 / == ``padding_idx`` are skipped) or as CSR (``ids``, ``offsets``).
* :func:`sparse_linear` -- BigDL ``SparseLinear``
  (``Zs/pipeline/api/keras/layers/SparseDense.scala:86-98``):
  ``y = X_sparse @ W^T + b`` with X a torch sparse COO/CSR tensor.

Parameter gradients accumulate in fp32 straight into the engine's flat gradient
buffer (like the conv/embedding kernels); the renorm factor of ``max_norm`` is a
constant in backward (an in-place renorm of the looked-up rows, as the
reference's LookupTable does). CPU tensors run the PyTorch reference below,
which doubles as the numerics oracle of ``tests/test_gpu_zoo_kernels.py``.
"""
import torch

from zoo.ops._native import native
from zoo.parallel.flat import grad_slot

_MODES = {"sum": 0, "mean": 1, "sqrtn": 2}


def _target(p):
    g = grad_slot(p)
    if g is not None:
        return g, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), False


def _ready(p):
    h = getattr(p, "_zoo_grad_ready", None)
    if h is not None:
        h(p)


# ---------------------------------------------------------------------------
# reference (CPU / oracle)
# ---------------------------------------------------------------------------
def embedding_bag_ref(table, ids, offsets=None, weights=None, combiner="sum", max_norm=-1.0, padding_idx=None):
    if offsets is None:
        B, L = ids.shape
        rows = torch.arange(B, device=ids.device).unsqueeze(1).expand(B, L).reshape(-1)
        ids = ids.reshape(-1)
        if weights is not None:
            weights = weights.reshape(-1)
    else:
        B = offsets.numel() - 1
        counts = offsets[1:] - offsets[:-1]
        rows = torch.repeat_interleave(torch.arange(B, device=ids.device), counts)
    ids = ids.long()
    keep = (ids >= 0) & (ids < table.shape[0])
    if padding_idx is not None:
        keep &= ids != int(padding_idx)
    rows, cols = rows[keep], ids[keep]
    w = torch.ones(cols.shape, dtype=table.dtype, device=table.device) if weights is None else \
        weights.reshape(-1)[keep].to(table.dtype)
    emb = table[cols]
    if max_norm is not None and max_norm > 0:
        n = emb.detach().norm(dim=1, keepdim=True)
        emb = emb * torch.where(n > max_norm, max_norm / (n + 1e-7), torch.ones_like(n))
    out = torch.zeros(B, table.shape[1], dtype=table.dtype, device=table.device).index_add(0, rows, emb * w[:, None])
    if combiner in ("mean", "sqrtn"):
        d = torch.zeros(B, dtype=table.dtype, device=table.device).index_add(0, rows, w if combiner == "mean" else w * w)
        d = d.clamp_min(1e-12)
        out = out / (d if combiner == "mean" else d.sqrt())[:, None]
    return out


# ---------------------------------------------------------------------------
# native
# ---------------------------------------------------------------------------
class _EmbeddingBagFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, ids, offsets, L, weights, mode, max_norm, pad):
        out, scale = native().embedding_bag_fwd(table.detach(), ids, offsets, L, weights, mode, max_norm, pad)
        ctx.save_for_backward(ids, offsets, weights, scale)
        ctx.table = table
        ctx.meta = (L, max_norm, pad)
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, offsets, weights, scale = ctx.saved_tensors
        L, max_norm, pad = ctx.meta
        table = ctx.table
        g, own = _target(table)
        native().embedding_bag_bwd(dout.float().contiguous(), table.detach(), ids, offsets, L, weights, scale, g,
                                   max_norm, pad)
        if own:
            _ready(table)
            return (None,) * 8
        return (g,) + (None,) * 7


def embedding_bag(table, ids, offsets=None, weights=None, combiner="sum", max_norm=-1.0, padding_idx=None):
    """[B, D] bag embeddings; ``ids`` [B, L] dense (``offsets`` None) or flat CSR ids."""
    if combiner not in _MODES:
        raise ValueError("combiner must be one of %s" % sorted(_MODES))
    if not table.is_cuda or table.dtype != torch.float32:
        return embedding_bag_ref(table, ids, offsets, weights, combiner, max_norm, padding_idx)
    ids = ids.long()
    if offsets is None:
        B, L = ids.shape
        flat_ids = ids.contiguous().reshape(-1)
        offs = torch.empty(0, dtype=torch.long, device=table.device)
    else:
        L = 0
        flat_ids = ids.contiguous().reshape(-1)
        offs = offsets.long().contiguous()
    w = None if weights is None else weights.float().contiguous().reshape(-1)
    pad = -1 if padding_idx is None else int(padding_idx)
    return _EmbeddingBagFn.apply(table, flat_ids, offs, int(L), w, _MODES[combiner],
                                 float(max_norm if max_norm is not None else -1.0), pad)


def coo_to_bags(x):
    """torch sparse [B, V] -> (ids, offsets, values) CSR bags (column ids per row)."""
    if x.layout == torch.sparse_csr:
        return x.col_indices(), x.crow_indices(), x.values()
    x = x.coalesce()
    rows, cols = x.indices()
    B = x.shape[0]
    offsets = torch.zeros(B + 1, dtype=torch.long, device=x.device)
    offsets[1:] = torch.bincount(rows, minlength=B).cumsum(0)
    return cols, offsets, x.values()


class _SparseLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, bias, crow, row, col, val):
        y = native().sparse_linear_fwd(crow, col, val, weight.detach(), None if bias is None else bias.detach())
        ctx.save_for_backward(row, col, val)
        ctx.weight, ctx.bias = weight, bias
        return y

    @staticmethod
    def backward(ctx, dy):
        row, col, val = ctx.saved_tensors
        w, b = ctx.weight, ctx.bias
        gw, own_w = _target(w)
        gb, own_b = (None, False) if b is None else _target(b)
        native().sparse_linear_bwd(row, col, val, dy.float().contiguous(), gw, gb)
        if own_w:
            _ready(w)
        if b is not None and own_b:
            _ready(b)
        return (None if own_w else gw, None if (b is None or own_b) else gb, None, None, None, None)


def sparse_linear(x, weight, bias=None):
    """``x`` sparse [B, IN] (COO or CSR) or dense; weight [O, IN]."""
    if not x.is_sparse and x.layout != torch.sparse_csr:
        return torch.nn.functional.linear(x, weight, bias)
    if not weight.is_cuda or weight.dtype != torch.float32:
        y = torch.sparse.mm(x.to_sparse_coo() if x.layout == torch.sparse_csr else x, weight.t())
        return y + bias if bias is not None else y
    cols, crow, vals = coo_to_bags(x)
    B = crow.numel() - 1
    rows = torch.repeat_interleave(torch.arange(B, device=x.device), crow[1:] - crow[:-1])
    return _SparseLinearFn.apply(weight, bias, crow.long().contiguous(), rows.long().contiguous(),
                                 cols.long().contiguous(), vals.float().contiguous())
