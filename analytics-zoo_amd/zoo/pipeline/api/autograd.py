"""Autograd API: math over symbolic Variables (and eager tensors).

Parity with Py/pipeline/api/autograd.py (568 LoC) and
Zs/pipeline/api/autograd/math.scala:32-611: ``mean, abs, sum, clip, square,
sqrt, exp, log, pow, maximum, neg, softsign, softplus, stack, expand_dims,
contiguous, mm, batch_dot, l2_normalize, erf, epsilon`` plus ``Variable``
operators, ``Parameter``, ``Constant``, ``Lambda`` and ``CustomLoss``.

Each function accepts either symbolic Variables (building a Lambda node of
the functional graph) or real tensors (evaluated immediately, so the same
expression code serves as the runtime body). Axis arguments follow the
reference: they count the batch dimension as axis 0.
"""
import numpy as np
import torch
import torch.nn as nn

from zoo.pipeline.api.keras.base import Lambda, Layer, NoBatchShape, Node, Variable, init_tensor, to_shape

EPS = 1e-7


def _lambda_node(fn, a, b=None, name="op"):
    if isinstance(b, Variable):
        return Lambda(lambda x, y: fn(x, y), name=None)([a, b])
    if b is None:
        return Lambda(lambda x: fn(x))(a)
    const = b

    def f(x):
        c = const
        if isinstance(c, (int, float)):
            return fn(x, c)
        return fn(x, torch.as_tensor(c, dtype=x.dtype, device=x.device))
    return Lambda(f)(a)


def _apply(fn, *args):
    args = tuple(_as_var(a) for a in args)
    if any(isinstance(a, Variable) for a in args):
        vs = [a for a in args if isinstance(a, Variable)]
        if len(vs) == 1 and len(args) == 1:
            return Lambda(lambda x: fn(x))(vs[0])
        idx = [i for i, a in enumerate(args) if isinstance(a, Variable)]
        consts = list(args)

        def f(*xs):
            full = list(consts)
            for i, x in zip(idx, xs):
                full[i] = x
            return fn(*full)
        return Lambda(f)(vs if len(vs) > 1 else vs[0])
    return fn(*args)


def _reduce(op, axis, keep):
    from zoo.ops.reduce import reduce   # native row reductions on the GPU (HK14)
    return lambda t: reduce(t, axis, op, keep)


def mean(x, axis=0, keepDims=False):  # noqa: N803 - reference name
    return _apply(_reduce("mean", axis, keepDims), x)


def abs(x):  # noqa: A001 - reference name
    return _apply(torch.abs, x)


def sum(x, axis=0, keepDims=False):  # noqa: A001,N803
    return _apply(_reduce("sum", axis, keepDims), x)


def clip(x, min, max):  # noqa: A002
    return _apply(lambda t: torch.clamp(t, min, max), x)


def square(x):
    return _apply(lambda t: t * t, x)


def sqrt(x):
    return _apply(torch.sqrt, x)


def exp(x):
    return _apply(torch.exp, x)


def log(x):
    return _apply(torch.log, x)


def pow(x, a):  # noqa: A001
    return _apply(lambda t: torch.pow(t, a), x)


def maximum(x, y):
    return _apply(torch.maximum, x, y)


def neg(x):
    return _apply(torch.neg, x)


def softsign(x):
    return _apply(lambda t: t / (1 + t.abs()), x)


def softplus(x):
    return _apply(torch.nn.functional.softplus, x)


def erf(x):
    return _apply(torch.erf, x)


def epsilon():
    return EPS


def contiguous(x):
    return _apply(lambda t: t.contiguous(), x)


def expand_dims(x, axis):
    return _apply(lambda t: t.unsqueeze(axis), x)


def stack(inputs, axis=1):
    inputs = [_as_var(v) for v in inputs]
    if any(isinstance(v, Variable) for v in inputs):
        return Lambda(lambda *xs: torch.stack(xs, dim=axis))(list(inputs))
    return torch.stack(inputs, dim=axis)


def l2_normalize(x, axis):
    from zoo.ops.reduce import l2_normalize as _l2   # native row kernel on the GPU (HK14)
    return _apply(lambda t: _l2(t, axis, EPS), x)


def mm(x, y, axes=None):
    """Matrix product of the last two dims (batched), optionally contracting
    ``axes=(ax_x, ax_y)`` (InternalMM, math.scala:258-315)."""
    def f(a, b):
        if axes is not None:
            ax_a, ax_b = axes
            if ax_a != a.dim() - 1:
                a = a.transpose(ax_a, a.dim() - 1)
            if ax_b != b.dim() - 2:
                b = b.transpose(ax_b, b.dim() - 2)
        from zoo.ops.bmm import bmm   # native batched GEMM on the GPU (HK2)
        return bmm(a, b)
    return _apply(f, x, y)


def batch_dot(x, y, axes=1, normalize=False):
    """Keras batch_dot over ``axes`` (math.scala:334)."""
    if isinstance(axes, int):
        axes = (axes, axes)

    def f(a, b):
        if normalize:
            a = a / torch.sqrt(torch.clamp((a * a).sum(dim=axes[0], keepdim=True), min=EPS))
            b = b / torch.sqrt(torch.clamp((b * b).sum(dim=axes[1], keepdim=True), min=EPS))
        if a.dim() == 2 and b.dim() == 2:
            return (a * b).sum(dim=1, keepdim=True)
        a2 = a.transpose(axes[0], -1) if axes[0] != a.dim() - 1 else a
        b2 = b.transpose(axes[1], 1) if axes[1] != 1 else b
        from zoo.ops.bmm import bmm   # native batched GEMM on the GPU (HK2)
        return bmm(a2, b2)
    return _apply(f, x, y)


class Parameter(Layer):
    """A trainable weight usable inside autograd expressions (KerasParameter.scala:31-208).

    Its value has exactly ``shape`` (no batch dimension)."""

    def __init__(self, shape, init_method=None, init_weight=None, trainable=True, name=None, **kwargs):
        super().__init__(name=name)
        self.p_shape = to_shape(shape)
        t = torch.empty(self.p_shape)
        if init_weight is not None:
            t.copy_(torch.as_tensor(np.asarray(init_weight), dtype=torch.float32).reshape(self.p_shape))
        else:
            init_tensor(t, init_method or "glorot_uniform")
        self.weight = nn.Parameter(t, requires_grad=trainable)
        self.built = True
        node = Node(self, [], [NoBatchShape(self.p_shape)])
        self.variable = node.outputs[0]

    def call(self, x=None):
        return self.weight

    def get_weight(self):
        return self.weight.detach().cpu().numpy()

    def set_weight(self, value):
        with torch.no_grad():
            self.weight.copy_(torch.as_tensor(np.asarray(value), dtype=self.weight.dtype))

    # arithmetic on the parameter's variable
    def __getattr__(self, item):
        try:
            return super().__getattr__(item)
        except AttributeError:
            return getattr(self.__dict__["variable"], item)

    def __add__(self, o):
        return self.variable + o

    def __radd__(self, o):
        return o + self.variable

    def __sub__(self, o):
        return self.variable - o

    def __rsub__(self, o):
        return o - self.variable

    def __mul__(self, o):
        return self.variable * o

    def __rmul__(self, o):
        return o * self.variable

    def __truediv__(self, o):
        return self.variable / o


class Constant(Layer):
    """A fixed tensor usable inside autograd expressions."""

    def __init__(self, data, name=None):
        super().__init__(name=name)
        self.register_buffer("value", torch.as_tensor(np.asarray(data), dtype=torch.float32))
        self.built = True
        node = Node(self, [], [NoBatchShape(self.value.shape)])
        self.variable = node.outputs[0]

    def call(self, x=None):
        return self.value


def _as_var(v):
    return v.variable if isinstance(v, (Parameter, Constant)) else v


class CustomLoss:
    """Loss from an autograd expression ``loss_func(y_true, y_pred)`` (CustomLoss.scala:29-126).
    The expression's per-sample values are averaged over the batch."""

    def __init__(self, loss_func, y_pred_shape, y_true_shape=None):
        from zoo.pipeline.api.keras.base import Input
        from zoo.pipeline.api.keras.engine.topology import Model
        y_true_shape = y_true_shape or y_pred_shape
        yt = Input(shape=y_true_shape)
        yp = Input(shape=y_pred_shape)
        out = loss_func(yt, yp)
        self.graph = Model([yt, yp], out)

    def __call__(self, y_pred, y_true):
        v = self.graph([y_true, y_pred])
        return v.mean()

    def forward(self, y_true, y_pred):
        return self(y_pred, y_true)
