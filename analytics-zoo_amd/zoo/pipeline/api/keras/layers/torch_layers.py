"""Shape / selection layers from the reference's torch.py and Scala layers:
Select, Narrow, Squeeze, SelectTable, Expand (+InternalExpand), SplitTensor
(+InternalSplitTensor), Softmax (+InternalSoftmax), ExpandDim, Recurrent.

Dimension arguments count the batch dimension as 0 (reference semantics).
"""
import torch

from zoo.pipeline.api.keras.base import Layer, to_shape


class Select(Layer):
    def __init__(self, dim, index, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim, self.index = int(dim), int(index)

    def compute_output_shape(self, s):
        s = list(s)
        del s[self.dim]
        return tuple(s)

    def call(self, x):
        return x.select(self.dim, self.index if self.index >= 0 else x.shape[self.dim] + self.index)


class Narrow(Layer):
    def __init__(self, dim, offset, length=1, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim, self.offset, self.length = int(dim), int(offset), int(length)

    def _len(self, size):
        off = self.offset if self.offset >= 0 else size + self.offset
        return (size - off) if self.length == -1 else (self.length if self.length > 0 else size - off + self.length + 1)

    def compute_output_shape(self, s):
        s = list(s)
        if s[self.dim] is not None:
            s[self.dim] = self._len(s[self.dim])
        return tuple(s)

    def call(self, x):
        size = x.shape[self.dim]
        off = self.offset if self.offset >= 0 else size + self.offset
        return x.narrow(self.dim, off, self._len(size))


class Squeeze(Layer):
    def __init__(self, dim=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dims = None if dim is None else ((dim,) if isinstance(dim, int) else tuple(dim))

    def compute_output_shape(self, s):
        if self.dims is None:
            return (None,) + tuple(d for d in s[1:] if d != 1)
        return tuple(d for i, d in enumerate(s) if i not in self.dims)

    def call(self, x):
        if self.dims is None:
            return x.reshape((x.shape[0],) + tuple(d for d in x.shape[1:] if d != 1))
        for d in sorted(self.dims, reverse=True):
            x = x.squeeze(d)
        return x


class SelectTable(Layer):
    def __init__(self, index, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.index = int(index)

    def compute_output_shape(self, s):
        return s[self.index]

    def call(self, xs):
        return xs[self.index]


class Expand(Layer):
    """Broadcast singleton dims to ``tgt_sizes`` (excl. batch; -1 keeps)."""

    def __init__(self, tgt_sizes, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.tgt = to_shape(tgt_sizes)

    def compute_output_shape(self, s):
        return (None,) + tuple(o if t == -1 else t for o, t in zip(s[1:], self.tgt))

    def call(self, x):
        return x.expand((x.shape[0],) + tuple(-1 if t == -1 else t for t in self.tgt))


class SplitTensor(Layer):
    """Split along ``dimension`` into ``num`` equal parts (a table output)."""

    def __init__(self, dimension, num, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dimension, self.num = int(dimension), int(num)

    def compute_output_shape(self, s):
        s = list(s)
        s[self.dimension] = s[self.dimension] // self.num
        return [tuple(s)] * self.num

    def call(self, x):
        return list(torch.chunk(x, self.num, dim=self.dimension))


class Softmax(Layer):
    """Softmax over the last dimension (max-shifted, InternalSoftmax)."""

    def call(self, x):
        from zoo.ops.nn import softmax
        return softmax(x, -1)


class Recurrent(Layer):
    """Generic recurrence container: applies ``cell(x_t, h) -> h`` over time."""

    def __init__(self, cell=None, return_sequences=False, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.cell, self.return_sequences = cell, return_sequences

    def call(self, x):
        h = None
        outs = []
        for t in range(x.shape[1]):
            h = self.cell(x[:, t], h)
            outs.append(h if not isinstance(h, (tuple, list)) else h[0])
        return torch.stack(outs, 1) if self.return_sequences else outs[-1]
