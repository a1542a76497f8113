"""Wide & Deep (Zs/models/recommendation/WideAndDeep.scala:54-365, Py wide_and_deep.py:29-239).

Wide part: a linear model over the (base + crossed) categorical columns. The
reference feeds a sparse multi-hot tensor to ``SparseDense``; here the wide
input is the per-column GLOBAL index (column offset + value), ``[batch,
n_wide_cols]`` int, and the linear layer is an embedding-bag sum over the
weight rows (SparseEmbedding, the HK10 gather) — the same math without
materialising a [batch, sum(wide_dims)] multi-hot matrix in HBM.
Deep part: multi-hot indicator columns + per-column embeddings +
continuous columns -> MLP. ``model_type`` in {wide, deep, wide_n_deep}.
"""
import torch

from zoo.models.recommendation.recommender import Recommender
from zoo.ops.wnd import deep_input, wnd_head
from zoo.pipeline.api.keras.base import Layer, init_tensor
from zoo.pipeline.api.keras.engine.topology import Model
from zoo.pipeline.api.keras.layers import Dense, Input, SparseEmbedding


class ColumnFeatureInfo:
    def __init__(self, wide_base_cols=None, wide_base_dims=None, wide_cross_cols=None, wide_cross_dims=None,
                 indicator_cols=None, indicator_dims=None, embed_cols=None, embed_in_dims=None, embed_out_dims=None,
                 continuous_cols=None, label="label"):
        self.wide_base_cols = list(wide_base_cols or [])
        self.wide_base_dims = [int(d) for d in (wide_base_dims or [])]
        self.wide_cross_cols = list(wide_cross_cols or [])
        self.wide_cross_dims = [int(d) for d in (wide_cross_dims or [])]
        self.indicator_cols = list(indicator_cols or [])
        self.indicator_dims = [int(d) for d in (indicator_dims or [])]
        self.embed_cols = list(embed_cols or [])
        self.embed_in_dims = [int(d) for d in (embed_in_dims or [])]
        self.embed_out_dims = [int(d) for d in (embed_out_dims or [])]
        self.continuous_cols = list(continuous_cols or [])
        self.label = label

    def __str__(self):
        return ("ColumnFeatureInfo {wide_base_cols: %s, wide_base_dims: %s, wide_cross_cols: %s, wide_cross_dims: %s, "
                "indicator_cols: %s, indicator_dims: %s, embed_cols: %s, embed_in_dims: %s, embed_out_dims: %s, "
                "continuous_cols: %s, label: '%s'}" % (
                    self.wide_base_cols, self.wide_base_dims, self.wide_cross_cols, self.wide_cross_dims,
                    self.indicator_cols, self.indicator_dims, self.embed_cols, self.embed_in_dims,
                    self.embed_out_dims, self.continuous_cols, self.label))


class DeepColumns(Layer):
    """The deep tower's input row: [indicator multi-hot | embedding(id_0) | ... | continuous]
    (WideAndDeep.scala:122-135: Select + LookupTable per embed column, JoinTable). One native
    kernel gathers the embedding rows (float ids converted in the kernel) and writes the whole
    row as the bf16 MFMA operand of the first Dense (zoo.ops.wnd.deep_input, csrc/kernels/wnd.hip);
    the table gradients are scatter-added straight into the flat gradient. Input: the list of
    present column groups in the order (indicator, embed ids, continuous)."""

    def __init__(self, indicator_dim=0, embed_in_dims=(), embed_out_dims=(), continuous_dim=0, init="normal",
                 **kwargs):
        super().__init__(**kwargs)
        self.indicator_dim, self.continuous_dim = int(indicator_dim), int(continuous_dim)
        self.embed_in_dims = [int(d) for d in embed_in_dims]
        self.embed_out_dims = [int(d) for d in embed_out_dims]
        self.init = init

    def build(self, input_shape):
        for i, (din, dout) in enumerate(zip(self.embed_in_dims, self.embed_out_dims)):
            w = torch.empty(din + 1, dout)          # ids are 1-based: row 0 stays unused, as LookupTable
            init_tensor(w, self.init)
            self.register_parameter("embeddings_%d" % i, torch.nn.Parameter(w))

    def compute_output_shape(self, input_shape):
        return (None, self.indicator_dim + sum(self.embed_out_dims) + self.continuous_dim)

    def call(self, xs):
        xs = list(xs) if isinstance(xs, (list, tuple)) else [xs]
        segs, ids = [], None
        k = 0
        if self.indicator_dim:
            segs.append(("dense", xs[k]))
            k += 1
        if self.embed_in_dims:
            ids = xs[k]
            k += 1
            for i in range(len(self.embed_in_dims)):
                segs.append(("embed", getattr(self, "embeddings_%d" % i), i))
        if self.continuous_dim:
            segs.append(("dense", xs[k]))
        if ids is None:
            ids = xs[0].new_zeros(xs[0].shape[0], 1)
        return deep_input(ids, segs)


class WideDeepHead(Layer):
    """softmax(wide + bias + deep): the wide tower's CAdd bias, the CAddTable merge and the final
    SoftMax of WideAndDeep.scala:136-144 in one native pass each way (zoo.ops.wnd.wnd_head).
    Input: [wide, deep], [wide] (with bias) or [deep] (no bias)."""

    def __init__(self, class_num, wide=True, deep=True, **kwargs):
        super().__init__(**kwargs)
        self.class_num, self.has_wide, self.has_deep = int(class_num), bool(wide), bool(deep)

    def build(self, input_shape):
        if self.has_wide:
            self.bias = torch.nn.Parameter(torch.zeros(self.class_num))

    def compute_output_shape(self, input_shape):
        return (None, self.class_num)

    def call(self, xs):
        xs = list(xs) if isinstance(xs, (list, tuple)) else [xs]
        wide = xs[0] if self.has_wide else None
        deep = xs[-1] if self.has_deep else None
        return wnd_head(wide, deep, self.bias if self.has_wide else None)


class WideAndDeep(Recommender):
    def __init__(self, class_num, column_info, model_type="wide_n_deep", hidden_layers=(40, 20, 10), **kwargs):
        super().__init__(**kwargs)
        ci = column_info
        if len(ci.wide_base_cols) != len(ci.wide_base_dims) or len(ci.wide_cross_cols) != len(ci.wide_cross_dims):
            raise ValueError("size of wide columns and dims should match")
        if len(ci.indicator_cols) != len(ci.indicator_dims):
            raise ValueError("size of indicator columns and dims should match")
        if not (len(ci.embed_cols) == len(ci.embed_in_dims) == len(ci.embed_out_dims)):
            raise ValueError("size of embed columns and dims should match")
        if model_type not in ("wide", "deep", "wide_n_deep"):
            raise TypeError("Unsupported model_type: %s" % model_type)
        self.class_num = int(class_num)
        self.column_info = ci
        self.model_type = model_type
        self.hidden_layers = [int(u) for u in hidden_layers]
        self._init_model()

    def _wide(self):
        ci = self.column_info
        n = len(ci.wide_base_cols) + len(ci.wide_cross_cols)
        dims = sum(ci.wide_base_dims) + sum(ci.wide_cross_dims)
        inp = Input(shape=(n,))
        return inp, SparseEmbedding(dims, self.class_num, combiner="sum", init="zero")(inp)

    def _deep(self):
        ci = self.column_info
        inputs = []
        if ci.indicator_dims:
            inputs.append(Input(shape=(sum(ci.indicator_dims),)))
        if ci.embed_in_dims:
            inputs.append(Input(shape=(len(ci.embed_in_dims),)))
        if ci.continuous_cols:
            inputs.append(Input(shape=(len(ci.continuous_cols),)))
        if not inputs:
            raise TypeError("Empty deep tensors")
        h = DeepColumns(sum(ci.indicator_dims), ci.embed_in_dims, ci.embed_out_dims, len(ci.continuous_cols))(
            inputs if len(inputs) > 1 else inputs[0])
        for u in self.hidden_layers:
            h = Dense(u, activation="relu")(h)
        return inputs, Dense(self.class_num, activation="relu")(h)

    def build_model(self):
        if self.model_type == "wide":
            inp, lin = self._wide()
            return Model(inp, WideDeepHead(self.class_num, wide=True, deep=False)(lin))
        if self.model_type == "deep":
            ins, deep = self._deep()
            return Model(ins if len(ins) > 1 else ins[0], WideDeepHead(self.class_num, wide=False, deep=True)(deep))
        winp, wide = self._wide()
        ins, deep = self._deep()
        return Model([winp] + ins, WideDeepHead(self.class_num)([wide, deep]))
