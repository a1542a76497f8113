"""NeuralCF (Zs/models/recommendation/NeuralCF.scala:45-138, Py neuralcf.py).

MLP tower over concatenated user/item embeddings + optional matrix
factorisation (element-wise product of a second pair of embeddings), concat,
Dense(num_classes, softmax). Embedding lookups run on the native gather /
scatter-add kernels, 8-aligned Dense layers on the MFMA GEMM.

``row_sparse_sync=True`` (or ``ZOO_ROW_SPARSE_SYNC=1``) makes data-parallel training
reduce the embedding-table gradients over the union of looked-up rows only
(``zoo.parallel.ddp.mark_row_sparse``) instead of all-reducing the dense tables.

On the GPU the whole network runs as the fused NCF kernels (zoo.ops.ncf, csrc/kernels/ncf.hip:
one forward and one backward launch plus a small weight-gradient reduction) whenever the widths
fit the kernel's caps (the defaults do); ``neuralcf._NCF_FUSED = False`` forces the layer-by-layer
graph (comparisons).
"""
import os

_NCF_FUSED = True

import torch

from zoo.models.recommendation.recommender import Recommender
from zoo.pipeline.api.keras.engine.topology import Model, merge
from zoo.pipeline.api.keras.layers import Dense, Embedding, Flatten, Input, Select


class NeuralCF(Recommender):
    def __init__(self, user_count, item_count, class_num, user_embed=20, item_embed=20, hidden_layers=(40, 20, 10),
                 include_mf=True, mf_embed=20, row_sparse_sync=None, **kwargs):
        super().__init__(**kwargs)
        if row_sparse_sync is None:
            row_sparse_sync = os.environ.get("ZOO_ROW_SPARSE_SYNC", "0") == "1"
        self.row_sparse_sync = bool(row_sparse_sync)
        self.user_count, self.item_count, self.class_num = int(user_count), int(item_count), int(class_num)
        self.user_embed, self.item_embed = int(user_embed), int(item_embed)
        self.hidden_layers = [int(h) for h in hidden_layers]
        self.include_mf, self.mf_embed = include_mf, int(mf_embed)
        self._init_model()
        if self.row_sparse_sync:
            from zoo.parallel.ddp import mark_row_sparse_embeddings
            mark_row_sparse_embeddings(self)

    def build_model(self):
        inp = Input(shape=(2,))
        user = Flatten()(Select(1, 0)(inp))
        item = Flatten()(Select(1, 1)(inp))
        emb_u = Embedding(self.user_count + 1, self.user_embed, init="normal")
        emb_i = Embedding(self.item_count + 1, self.item_embed, init="normal")
        mlp_u = Flatten()(emb_u(user))
        mlp_i = Flatten()(emb_i(item))
        h = merge([mlp_u, mlp_i], mode="concat", concat_axis=1)
        dense = []
        for units in self.hidden_layers:
            dense.append(Dense(units, activation="relu"))
            h = dense[-1](h)
        emb_mu = emb_mi = None
        if self.include_mf:
            emb_mu = Embedding(self.user_count + 1, self.mf_embed, init="normal")
            emb_mi = Embedding(self.item_count + 1, self.mf_embed, init="normal")
            mf_u = Flatten()(emb_mu(user))
            mf_i = Flatten()(emb_mi(item))
            mf = merge([mf_u, mf_i], mode="mul", concat_axis=1)
            h = merge([h, mf], mode="concat", concat_axis=1)
        out_dense = Dense(self.class_num, activation="softmax")
        out = out_dense(h)
        # handles for the fused path, kept out of the module tree (same parameters, no new keys)
        self.__dict__["_ncf_parts"] = (emb_u, emb_i, emb_mu, emb_mi, dense, out_dense)
        return Model(inp, out)

    # ------------------------------------------------------------------ fused GPU path
    def _fused_dims(self, x):
        parts = self.__dict__.get("_ncf_parts")
        if parts is None or not _NCF_FUSED:
            return None
        if not (torch.is_tensor(x) and x.is_cuda and x.dim() == 2 and x.shape[1] == 2 and x.shape[0] > 0):
            return None
        emb_u, emb_i, emb_mu, emb_mi, dense, out_dense = parts
        if len(dense) != 3:
            return None
        embs = [e for e in (emb_u, emb_i, emb_mu, emb_mi) if e is not None]
        if any(e.mask_zero or not e.zero_based_id for e in embs):
            return None
        if any(not hasattr(e, "embeddings") or not e.embeddings.is_cuda for e in embs):
            return None
        dims = (self.user_embed, self.item_embed, self.mf_embed if self.include_mf else 0,
                dense[0].output_dim, dense[1].output_dim, dense[2].output_dim, self.class_num, 0)
        from zoo.ops.ncf import ncf_fused_ok
        return dims if ncf_fused_ok(dims) else None

    def forward(self, x, *rest):
        dims = None if rest else self._fused_dims(x)
        if dims is None:
            return super().forward(x, *rest)
        from zoo.ops.ncf import ncf_fused
        emb_u, emb_i, emb_mu, emb_mi, dense, out_dense = self.__dict__["_ncf_parts"]
        ids = x.long()
        tabs = [emb_u.embeddings, emb_i.embeddings, None if emb_mu is None else emb_mu.embeddings,
                None if emb_mi is None else emb_mi.embeddings]
        if self.row_sparse_sync:
            from zoo.parallel.ddp import record_lookup
            for t, col in zip(tabs, (0, 1, 0, 1)):
                if t is not None:
                    record_lookup(t, ids[:, col])
        return ncf_fused(ids, dims, *tabs, dense[0].weight, dense[0].bias, dense[1].weight, dense[1].bias,
                         dense[2].weight, dense[2].bias, out_dense.weight, out_dense.bias)
