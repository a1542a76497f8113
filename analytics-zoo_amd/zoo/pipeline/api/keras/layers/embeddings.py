"""Embedding layers: Embedding (LookupTable, Embedding.scala:82-100),
SparseEmbedding (LookupTableSparse with combiner, SparseEmbedding.scala:76-88)
and WordEmbedding (frozen pre-trained vectors, WordEmbedding.scala).

Lookups run on the native gather / scatter-add kernels (HK9).
Zoo Keras Embedding takes 0-based indices by default like Keras.
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.pipeline.api.keras.base import Layer, init_tensor


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, init="uniform", weights=None, trainable=True, input_length=None,
                 W_regularizer=None, input_shape=None, mask_zero=False, padding_value=0, zero_based_id=True,
                 **kwargs):
        if input_shape is None and input_length is not None:
            input_shape = (input_length,)
        super().__init__(input_shape=input_shape, **kwargs)
        self.input_dim, self.output_dim, self.init = int(input_dim), int(output_dim), init
        self.init_weights, self.trainable_w = weights, trainable
        self.mask_zero, self.zero_based_id = mask_zero, zero_based_id
        self.add_regularizer(W_regularizer, "embeddings")

    def build(self, input_shape):
        w = torch.empty(self.input_dim, self.output_dim)
        if self.init_weights is not None:
            w.copy_(torch.as_tensor(np.asarray(self.init_weights[0] if isinstance(self.init_weights, list)
                                               else self.init_weights), dtype=torch.float32))
        else:
            init_tensor(w, self.init)
        self.embeddings = nn.Parameter(w, requires_grad=self.trainable_w)

    def compute_output_shape(self, input_shape):
        return tuple(input_shape) + (self.output_dim,)

    def call(self, x):
        idx = x.long()
        if not self.zero_based_id:
            idx = idx - 1
        out = ops.embedding(idx, self.embeddings, padding_idx=0 if self.mask_zero else None)
        return out


class WordEmbedding(Embedding):
    """Embedding initialised from a GloVe-style text file (``word v1 v2 ...``)
    and frozen by default. ``word_index`` maps word -> index (1-based; index 0
    is reserved for unknown words)."""

    def __init__(self, embedding_file, word_index=None, trainable=False, input_length=None, input_shape=None,
                 **kwargs):
        vecs = {}
        dim = None
        with open(embedding_file, "r", encoding="utf-8") as f:
            for line in f:
                parts = line.rstrip().split(" ")
                if len(parts) < 2:
                    continue
                if word_index is None or parts[0] in word_index:
                    vecs[parts[0]] = np.asarray(parts[1:], dtype=np.float32)
                    dim = len(parts) - 1
        if word_index is None:
            word_index = {w: i + 1 for i, w in enumerate(sorted(vecs))}
        n = max(word_index.values()) + 1
        table = np.zeros((n, dim), dtype=np.float32)
        for w, i in word_index.items():
            if w in vecs:
                table[i] = vecs[w]
        self.word_index = word_index
        super().__init__(n, dim, weights=[table], trainable=trainable, input_length=input_length,
                         input_shape=input_shape, **kwargs)

    @staticmethod
    def get_word_index(embedding_file):
        idx = {}
        with open(embedding_file, "r", encoding="utf-8") as f:
            for i, line in enumerate(f):
                idx[line.split(" ", 1)[0]] = i + 1
        return idx


class SparseEmbedding(Layer):
    """Bag-of-ids embedding with ``combiner`` in {sum, mean, sqrtn}. Input is a
    dense id tensor [batch, n] where ids < 0 are padding (ignored), or a torch
    sparse COO tensor [batch, vocab] with the ids as column indices."""

    def __init__(self, input_dim, output_dim, combiner="sum", max_norm=-1.0, init="uniform", W_regularizer=None,
                 input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.input_dim, self.output_dim, self.combiner = int(input_dim), int(output_dim), combiner
        self.max_norm, self.init = max_norm, init

    def build(self, input_shape):
        self.embeddings = nn.Parameter(init_tensor(torch.empty(self.input_dim, self.output_dim), self.init))

    def compute_output_shape(self, input_shape):
        return (None, self.output_dim)

    def call(self, x):
        # native embedding-bag kernel on GPU (zoo/ops/sparse.py, csrc/kernels/sparse.hip)
        from zoo.ops.sparse import coo_to_bags, embedding_bag
        if x.is_sparse or x.layout == torch.sparse_csr:
            ids, offsets, vals = coo_to_bags(x)
            return embedding_bag(self.embeddings, ids, offsets, vals, self.combiner, self.max_norm)
        ids = x.long()
        if ids.dim() == 1:
            ids = ids.unsqueeze(1)
        return embedding_bag(self.embeddings, ids, None, None, self.combiner, self.max_norm)
