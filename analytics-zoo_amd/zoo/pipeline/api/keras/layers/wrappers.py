"""Layer wrappers: TimeDistributed (+InternalTimeDistributed), Bidirectional,
KerasLayerWrapper (Py/pipeline/api/keras/layers/wrappers.py)."""
import copy

import torch

from zoo.pipeline.api.keras.base import Layer


class TimeDistributed(Layer):
    """Apply ``layer`` to every temporal slice: [B, T, ...] -> layer([B*T, ...])."""

    def __init__(self, layer, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.layer = layer

    def build(self, input_shape):
        self.layer._ensure_built((None,) + tuple(input_shape[2:]))

    def compute_output_shape(self, input_shape):
        inner = self.layer.compute_output_shape((None,) + tuple(input_shape[2:]))
        return (None, input_shape[1]) + tuple(inner[1:])

    def call(self, x):
        B, T = x.shape[:2]
        y = self.layer(x.reshape(B * T, *x.shape[2:]))
        return y.reshape(B, T, *y.shape[1:])


class Bidirectional(Layer):
    """Run a recurrent layer forwards and backwards and merge (concat/sum/mul/ave)."""

    def __init__(self, layer, merge_mode="concat", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.forward_layer = layer
        self.backward_layer = copy.deepcopy(layer)
        self.backward_layer.name = layer.name + "_backward"
        self.backward_layer.go_backwards = not getattr(layer, "go_backwards", False)
        self.merge_mode = merge_mode

    def build(self, input_shape):
        self.forward_layer._ensure_built(input_shape)
        self.backward_layer._ensure_built(input_shape)

    def compute_output_shape(self, input_shape):
        s = self.forward_layer.compute_output_shape(input_shape)
        if self.merge_mode == "concat":
            return tuple(s[:-1]) + (2 * s[-1],)
        return s

    def call(self, x):
        a = self.forward_layer(x)
        b = self.backward_layer(x)
        if getattr(self.backward_layer, "return_sequences", False):
            b = torch.flip(b, dims=[1])
        m = self.merge_mode
        if m == "concat":
            return torch.cat([a, b], dim=-1)
        if m == "sum":
            return a + b
        if m == "mul":
            return a * b
        if m == "ave":
            return (a + b) / 2
        raise ValueError("Unsupported merge_mode %s" % m)


class KerasLayerWrapper(Layer):
    """Wrap any torch.nn.Module (the reference wraps a BigDL module)."""

    def __init__(self, torch_layer, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.module = torch_layer

    def compute_output_shape(self, input_shape):
        from zoo.pipeline.api.keras.base import _dummy
        with torch.no_grad():
            out = self.module(_dummy(input_shape))
        return (None,) + tuple(out.shape[1:])

    def call(self, x):
        return self.module(x)
