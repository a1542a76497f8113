"""NeuralCF (Zs/models/recommendation/NeuralCF.scala:45-138, Py neuralcf.py).

MLP tower over concatenated user/item embeddings + optional matrix
factorisation (element-wise product of a second pair of embeddings), concat,
Dense(num_classes, softmax). Embedding lookups run on the native gather /
scatter-add kernels, 8-aligned Dense layers on the MFMA GEMM.

``row_sparse_sync=True`` (or ``ZOO_ROW_SPARSE_SYNC=1``) makes data-parallel training
reduce the embedding-table gradients over the union of looked-up rows only
(``zoo.parallel.ddp.mark_row_sparse``) instead of all-reducing the dense tables.
"""
import os

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
        mlp_u = Flatten()(Embedding(self.user_count + 1, self.user_embed, init="normal")(user))
        mlp_i = Flatten()(Embedding(self.item_count + 1, self.item_embed, init="normal")(item))
        h = merge([mlp_u, mlp_i], mode="concat", concat_axis=1)
        for units in self.hidden_layers:
            h = Dense(units, activation="relu")(h)
        if self.include_mf:
            mf_u = Flatten()(Embedding(self.user_count + 1, self.mf_embed, init="normal")(user))
            mf_i = Flatten()(Embedding(self.item_count + 1, self.mf_embed, init="normal")(item))
            mf = merge([mf_u, mf_i], mode="mul", concat_axis=1)
            h = merge([h, mf], mode="concat", concat_axis=1)
        out = Dense(self.class_num, activation="softmax")(h)
        return Model(inp, out)
