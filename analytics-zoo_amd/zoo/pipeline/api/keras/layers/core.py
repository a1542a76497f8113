"""Core Keras layers (Py/pipeline/api/keras/layers/core.py; Zs keras layers
Dense.scala:97, SparseDense, MaxoutDense, Highway, Dropout, Flatten, Reshape,
Permute, RepeatVector, Masking, SpatialDropout1D/2D/3D, Activation, GetShape,
Max, ExpandDim).

Dense runs on the native MFMA GEMM (``zoo.ops.linear``) with bias and
relu/gelu/sigmoid/tanh fused in the epilogue when the feature sizes are
8-aligned; other sizes use the plain library GEMM.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.pipeline.api.keras.base import Layer, apply_activation, check_activation, init_tensor, to_shape

_FUSABLE = {None, "linear", "relu", "gelu", "sigmoid", "tanh"}


class Dense(Layer):
    def __init__(self, output_dim, init="glorot_uniform", limits=None, activation=None, W_regularizer=None,
                 b_regularizer=None, bias=True, input_dim=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, input_dim=input_dim, **kwargs)
        self.output_dim = int(output_dim)
        self.init, self.limits = init, limits
        self.activation = check_activation(activation)
        self.use_bias = bias
        self.add_regularizer(W_regularizer, "weight")
        self.add_regularizer(b_regularizer, "bias")

    def build(self, input_shape):
        d = input_shape[-1]
        self.weight = nn.Parameter(init_tensor(torch.empty(self.output_dim, d), self.init, limits=self.limits))
        self.bias = nn.Parameter(torch.zeros(self.output_dim)) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        return tuple(input_shape[:-1]) + (self.output_dim,)

    def call(self, x):
        act = self.activation if (isinstance(self.activation, str) and self.activation.lower() in _FUSABLE) \
            or self.activation is None else None
        y = ops.linear(x, self.weight, self.bias, act=act.lower() if isinstance(act, str) else None)
        if act is None and self.activation is not None:
            y = apply_activation(y, self.activation)
        return y


class Activation(Layer):
    def __init__(self, activation, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.activation = check_activation(activation)

    def call(self, x):
        return apply_activation(x, self.activation)


class Dropout(Layer):
    def __init__(self, p, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.p = float(p)

    def call(self, x):
        from zoo.ops.pointwise import dropout   # native counter-hash mask on the GPU (HK16)
        return dropout(x, self.p, self.training)


class SpatialDropout1D(Layer):
    """Drops whole feature maps of (batch, steps, channels)."""

    def __init__(self, p=0.5, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.p = float(p)

    def call(self, x):
        if not self.training or self.p == 0:
            return x
        mask = (torch.rand(x.shape[0], 1, x.shape[2], device=x.device) >= self.p).to(x.dtype) / (1 - self.p)
        return x * mask


class SpatialDropout2D(Layer):
    def __init__(self, p=0.5, dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.p, self.dim_ordering = float(p), dim_ordering

    def call(self, x):
        if not self.training or self.p == 0:
            return x
        if self.dim_ordering == "th":
            shape = (x.shape[0], x.shape[1]) + (1,) * (x.dim() - 2)
        else:
            shape = (x.shape[0],) + (1,) * (x.dim() - 2) + (x.shape[-1],)
        mask = (torch.rand(shape, device=x.device) >= self.p).to(x.dtype) / (1 - self.p)
        return x * mask


class SpatialDropout3D(SpatialDropout2D):
    pass


class Flatten(Layer):
    def compute_output_shape(self, input_shape):
        return (None, int(np.prod(input_shape[1:])))

    def call(self, x):
        return x.reshape(x.shape[0], -1)


class Reshape(Layer):
    def __init__(self, target_shape, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.target_shape = to_shape(target_shape)

    def _resolve(self, in_shape):
        tgt = list(self.target_shape)
        if -1 in tgt:
            known = int(np.prod([d for d in tgt if d != -1]))
            total = int(np.prod(in_shape[1:]))
            tgt[tgt.index(-1)] = total // known
        return tuple(tgt)

    def compute_output_shape(self, input_shape):
        return (None,) + self._resolve(input_shape)

    def call(self, x):
        return x.reshape((x.shape[0],) + self._resolve((None,) + tuple(x.shape[1:])))


class Permute(Layer):
    """dims are 1-based and exclude the batch axis (Keras 1)."""

    def __init__(self, dims, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dims = tuple(dims)

    def compute_output_shape(self, input_shape):
        return (None,) + tuple(input_shape[d] for d in self.dims)

    def call(self, x):
        return x.permute((0,) + self.dims)


class RepeatVector(Layer):
    def __init__(self, n, input_dim=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, input_dim=input_dim, **kwargs)
        self.n = int(n)

    def compute_output_shape(self, input_shape):
        return (None, self.n, input_shape[-1])

    def call(self, x):
        return x.unsqueeze(1).expand(x.shape[0], self.n, x.shape[-1])


class Masking(Layer):
    """Zero out timesteps whose features all equal ``mask_value``."""

    def __init__(self, mask_value=0.0, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.mask_value = float(mask_value)

    def call(self, x):
        keep = (x != self.mask_value).any(dim=-1, keepdim=True)
        return x * keep.to(x.dtype)


class GetShape(Layer):
    def compute_output_shape(self, input_shape):
        return (None, len(input_shape) - 1)

    def call(self, x):
        s = torch.tensor(list(x.shape[1:]), dtype=torch.float32, device=x.device)
        return s.unsqueeze(0).expand(x.shape[0], -1)


class SparseDense(Layer):
    """Dense layer for sparse input (SparseDense.scala:86-98). Accepts a torch
    sparse COO tensor or a dense tensor; backward w.r.t. the (sparse) input is
    skipped when ``backward_start``/``backward_length`` is -1 like the reference."""

    def __init__(self, output_dim, init="glorot_uniform", activation=None, W_regularizer=None,
                 b_regularizer=None, backward_start=-1, backward_length=-1, init_weight=None, init_bias=None,
                 bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.output_dim, self.init, self.activation, self.use_bias = int(output_dim), init, activation, bias
        self.init_weight, self.init_bias = init_weight, init_bias
        self.add_regularizer(W_regularizer, "weight")
        self.add_regularizer(b_regularizer, "bias")

    def build(self, input_shape):
        d = input_shape[-1]
        w = torch.empty(self.output_dim, d)
        if self.init_weight is not None:
            w.copy_(torch.as_tensor(np.asarray(self.init_weight)).reshape(w.shape))
        else:
            init_tensor(w, self.init)
        self.weight = nn.Parameter(w)
        b = torch.zeros(self.output_dim)
        if self.init_bias is not None:
            b.copy_(torch.as_tensor(np.asarray(self.init_bias)))
        self.bias = nn.Parameter(b) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        return (None, self.output_dim)

    def call(self, x):
        # CSR/COO input runs the native sparse-linear kernel on GPU (zoo/ops/sparse.py)
        from zoo.ops.sparse import sparse_linear
        return apply_activation(sparse_linear(x, self.weight, self.bias), self.activation)


class MaxoutDense(Layer):
    def __init__(self, output_dim, nb_feature=4, W_regularizer=None, b_regularizer=None, bias=True,
                 input_dim=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, input_dim=input_dim, **kwargs)
        self.output_dim, self.nb_feature, self.use_bias = int(output_dim), int(nb_feature), bias
        self.add_regularizer(W_regularizer, "weight")

    def build(self, input_shape):
        d = input_shape[-1]
        self.weight = nn.Parameter(init_tensor(torch.empty(self.output_dim * self.nb_feature, d), "glorot_uniform"))
        self.bias = nn.Parameter(torch.zeros(self.output_dim * self.nb_feature)) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        return (None, self.output_dim)

    def call(self, x):
        y = ops.linear(x, self.weight, self.bias)
        return y.reshape(x.shape[0], self.nb_feature, self.output_dim).max(dim=1).values


class Highway(Layer):
    """y = t * h(W x) + (1 - t) * x with transform gate t = sigmoid(W_t x)."""

    def __init__(self, activation=None, W_regularizer=None, b_regularizer=None, bias=True, input_dim=None,
                 input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, input_dim=input_dim, **kwargs)
        self.activation, self.use_bias = activation, bias

    def build(self, input_shape):
        d = input_shape[-1]
        self.weight = nn.Parameter(init_tensor(torch.empty(2 * d, d), "glorot_uniform"))
        b = torch.zeros(2 * d)
        b[d:] = -2.0  # carry-biased transform gate
        self.bias = nn.Parameter(b) if self.use_bias else None

    def call(self, x):
        d = x.shape[-1]
        y = ops.linear(x, self.weight, self.bias)
        h = apply_activation(y[..., :d], self.activation)
        t = torch.sigmoid(y[..., d:])
        return t * h + (1 - t) * x


class Max(Layer):
    """Max over ``dim`` (1-based incl. batch? reference: dim excludes batch)."""

    def __init__(self, dim, num_input_dims=-2147483648, return_value=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim, self.return_value = int(dim), return_value

    def compute_output_shape(self, input_shape):
        s = list(input_shape)
        del s[self.dim]
        return tuple(s)

    def call(self, x):
        r = x.max(dim=self.dim)
        return r.values if self.return_value else r.indices.to(x.dtype)


class ExpandDim(Layer):
    def __init__(self, dim, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim = int(dim)

    def compute_output_shape(self, input_shape):
        s = list(input_shape)
        s.insert(self.dim, 1)
        return tuple(s)

    def call(self, x):
        return x.unsqueeze(self.dim)
