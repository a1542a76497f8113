"""Keras-1 style layer base, symbolic graph (Variable/Node) and helpers.

Parity: ``ZooKerasLayer`` (Py/pipeline/api/keras/base.py:83-122), shape
inference (``InferShape``), ``get/set_weights``, the functional API where
calling a layer on a Variable creates a graph node (Zs KerasLayer/Node), and
the init / activation string tables of KerasUtils.scala:39-176.

Every layer is a ``torch.nn.Module``; running a model executes the layers'
``call`` on real tensors, which dispatch to the native gfx950 kernels
(``zoo.ops``) on the GPU. Shapes follow Keras: tuples whose first entry is the
batch dimension ``None``.
"""
import itertools
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

_uid = itertools.count()


def _auto_name(obj):
    return "%s%d" % (type(obj).__name__.lower(), next(_uid))


class NoBatchShape(tuple):
    """Shape of a graph value that has no batch dimension (Parameter / Constant)."""
    no_batch = True


def to_shape(s):
    if s is None:
        return None
    if isinstance(s, int):
        return (s,)
    if isinstance(s, tuple):
        return s
    return tuple(s)


# ----------------------------------------------------------------------------
# initializers (KerasUtils.getInitMethod)
# ----------------------------------------------------------------------------
def _fans(shape, fan_in=None, fan_out=None):
    if fan_in is not None:
        return fan_in, fan_out
    if len(shape) == 2:
        return shape[1], shape[0]
    rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    return shape[1] * rf, shape[0] * rf


def init_tensor(t, method, fan_in=None, fan_out=None, limits=None):
    method = (method or "glorot_uniform").lower() if isinstance(method, str) else method
    with torch.no_grad():
        if callable(method):
            t.copy_(torch.as_tensor(method(tuple(t.shape)), dtype=t.dtype))
            return t
        fi, fo = _fans(tuple(t.shape), fan_in, fan_out)
        if method in ("glorot_uniform", "xavier"):
            a = math.sqrt(6.0 / (fi + fo))
            t.uniform_(-a, a)
        elif method == "glorot_normal":
            t.normal_(0.0, math.sqrt(2.0 / (fi + fo)))
        elif method in ("one", "ones"):
            t.fill_(1.0)
        elif method in ("zero", "zeros"):
            t.zero_()
        elif method == "uniform":
            lo, hi = limits if limits else (-0.05, 0.05)
            t.uniform_(lo, hi)
        elif method == "normal":
            mean, std = limits if limits else (0.0, 0.05)
            t.normal_(mean, std)
        elif method == "he_normal":
            t.normal_(0.0, math.sqrt(2.0 / fi))
        elif method == "he_uniform":
            a = math.sqrt(6.0 / fi)
            t.uniform_(-a, a)
        elif method == "lecun_uniform":
            a = math.sqrt(3.0 / fi)
            t.uniform_(-a, a)
        elif method == "identity":
            t.zero_()
            n = min(t.shape[0], t.shape[1])
            t[:n, :n] = torch.eye(n)
        else:
            raise ValueError("Unsupported init method: %s" % method)
    return t


# ----------------------------------------------------------------------------
# activations (KerasUtils.getKerasActivation)
# ----------------------------------------------------------------------------
def hard_sigmoid(x):
    return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)


_ACTS = {
    "tanh": torch.tanh, "sigmoid": torch.sigmoid, "relu": torch.relu, "softmax": None,
    "softplus": F.softplus, "softsign": F.softsign, "hard_sigmoid": hard_sigmoid, "relu6": F.relu6,
    "tanh_shrink": F.tanhshrink, "softmin": None, "log_sigmoid": F.logsigmoid, "log_softmax": None,
    "linear": lambda x: x, "gelu": F.gelu, "elu": F.elu, "selu": F.selu, "exponential": torch.exp,
    "swish": F.silu,
}


def apply_activation(x, name):
    if name is None:
        return x
    if callable(name):
        return name(x)
    n = name.lower()
    if n in ("softmax", "softmin", "log_softmax"):
        from zoo.ops.nn import softmax  # native row kernel on the GPU
        if n == "softmax":
            return softmax(x, -1 if x.dim() != 4 else 1)
        if n == "softmin":
            return softmax(-x, -1)
        return softmax(x, -1, log=True)
    if n not in _ACTS:
        raise ValueError("Unsupported activation: %s" % name)
    if x.is_cuda and n not in ("linear",):
        from zoo.ops.pointwise import ACT_CODES, activation   # native fwd/bwd kernels (HK13)
        if n in ACT_CODES:
            return activation(x, n)
    return _ACTS[n](x)


def check_activation(name):
    if name is not None and not callable(name) and name.lower() not in _ACTS:
        raise ValueError("Unsupported activation: %s" % name)
    return name


# ----------------------------------------------------------------------------
# regularizers (Py/pipeline/api/keras/regularizers.py -> BigDL L1/L2)
# ----------------------------------------------------------------------------
class Regularizer:
    def __init__(self, l1=0.0, l2=0.0):
        self.l1, self.l2 = float(l1), float(l2)

    def __call__(self, w):
        r = 0.0
        if self.l1:
            r = r + self.l1 * w.abs().sum()
        if self.l2:
            r = r + self.l2 * (w * w).sum()
        return r


def l1(l=0.01):
    return Regularizer(l1=l)


def l2(l=0.01):
    return Regularizer(l2=l)


def l1l2(l1=0.01, l2=0.01):  # noqa: F811 - keras name
    return Regularizer(l1=l1, l2=l2)


# ----------------------------------------------------------------------------
# symbolic graph
# ----------------------------------------------------------------------------
class Node:
    """One application of a layer to symbolic inputs."""

    def __init__(self, layer, inputs, output_shapes):
        self.layer = layer
        self.inputs = inputs            # list[Variable]
        self.output_shapes = output_shapes
        self.outputs = [Variable(self, i, s) for i, s in enumerate(output_shapes)]


class Variable:
    """Symbolic tensor in a functional graph (Py/pipeline/api/autograd.py:369).

    Supports the autograd operator set (``+ - * /``, ``**``, indexing, ...)
    which create Lambda nodes, so custom losses / layers can be written as
    expressions over Variables.
    """

    def __init__(self, node, index=0, shape=None, name=None):
        self.node = node
        self.index = index
        self.shape = to_shape(shape)
        self.name = name

    # keras-ish helpers
    def get_output_shape(self):
        return self.shape

    def get_input_shape(self):
        return self.shape

    @property
    def ndim(self):
        return len(self.shape)

    # ------ operators -> Lambda nodes (implemented in autograd.py) ---------
    def _op(self, fn, other=None, name="op"):
        from zoo.pipeline.api.autograd import _lambda_node, _as_var
        return _lambda_node(fn, self, _as_var(other), name)

    def __add__(self, o):
        return self._op(lambda a, b: a + b, o, "add")

    def __radd__(self, o):
        return self._op(lambda a, b: b + a, o, "radd")

    def __sub__(self, o):
        return self._op(lambda a, b: a - b, o, "sub")

    def __rsub__(self, o):
        return self._op(lambda a, b: b - a, o, "rsub")

    def __mul__(self, o):
        return self._op(lambda a, b: a * b, o, "mul")

    def __rmul__(self, o):
        return self._op(lambda a, b: b * a, o, "rmul")

    def __truediv__(self, o):
        return self._op(lambda a, b: a / b, o, "div")

    def __rtruediv__(self, o):
        return self._op(lambda a, b: b / a, o, "rdiv")

    __div__ = __truediv__
    __rdiv__ = __rtruediv__

    def __neg__(self):
        return self._op(lambda a: -a, None, "neg")

    def __pow__(self, a):
        return self._op(lambda x: x ** a, None, "pow")

    def __getitem__(self, idx):
        return self._op(lambda x: x[(slice(None),) + (idx if isinstance(idx, tuple) else (idx,))], None, "slice")

    def slice(self, dim, start_index, length):
        return self._op(lambda x: x.narrow(dim, start_index, length), None, "narrow")

    def index_select(self, dim, index):
        return self._op(lambda x: x.select(dim, index), None, "select")

    def squeeze(self, dim=None):
        return self._op(lambda x: x.squeeze(dim) if dim is not None else x.squeeze(), None, "squeeze")


def _flatten_vars(x):
    if isinstance(x, Variable):
        return [x]
    if isinstance(x, (list, tuple)):
        out = []
        for e in x:
            out.extend(_flatten_vars(e))
        return out
    return []


def is_symbolic(x):
    if isinstance(x, Variable):
        return True
    return isinstance(x, (list, tuple)) and len(x) > 0 and all(isinstance(e, Variable) for e in x)


class Layer(nn.Module):
    """Base class of every zoo Keras layer (ZooKerasLayer)."""

    def __init_subclass__(cls, **kw):
        # record constructor arguments (outermost __init__ only) for save/load
        super().__init_subclass__(**kw)
        orig = cls.__init__  # own or inherited (an inherited wrapper skips itself)

        def init(self, *a, **k):
            if "_init_args" not in self.__dict__:
                object.__setattr__(self, "_init_args", (cls, a, dict(k)))
            orig(self, *a, **k)
        init.__doc__ = orig.__doc__
        init.__wrapped__ = orig
        cls.__init__ = init

    def __init__(self, input_shape=None, name=None, input_dim=None, **kwargs):
        super().__init__()
        if input_shape is None and input_dim is not None:
            input_shape = (input_dim,)
        self._given_input_shape = to_shape(input_shape)
        self.name = name or _auto_name(self)
        self.built = False
        self._input_shape = None
        self._output_shape = None
        self.trainable = True
        self._regularizers = []

    # ---- to override ------------------------------------------------------
    def build(self, input_shape):
        """Create weights; ``input_shape`` includes the batch entry (None)."""

    def compute_output_shape(self, input_shape):
        return input_shape

    def call(self, x):
        raise NotImplementedError

    # ---- machinery ----------------------------------------------------------
    def _ensure_built(self, input_shape):
        if not self.built:
            self.build(input_shape)
            self.built = True
            self._input_shape = input_shape
            self._output_shape = self.compute_output_shape(input_shape)

    @staticmethod
    def _runtime_shape(x):
        if isinstance(x, (list, tuple)):
            return [Layer._runtime_shape(e) for e in x]
        return (None,) + tuple(x.shape[1:])

    def forward(self, x, *rest):
        if rest:
            x = [x] + list(rest)
        if not self.built:
            self._ensure_built(self._runtime_shape(x))
        return self.call(x)

    def __call__(self, *args, **kw):
        x = args[0] if len(args) == 1 else list(args)
        if is_symbolic(x):
            return self._symbolic(x)
        return super().__call__(*args, **kw)

    def _symbolic(self, x):
        shapes = [v.shape for v in x] if isinstance(x, (list, tuple)) else x.shape
        if not self.built:
            self._ensure_built(shapes)
        out_shape = self.compute_output_shape(shapes)
        multi = isinstance(out_shape, list)
        node = Node(self, list(x) if isinstance(x, (list, tuple)) else [x], out_shape if multi else [out_shape])
        node.list_input = isinstance(x, (list, tuple))
        return node.outputs if multi else node.outputs[0]

    def build_from_input_shape(self):
        if self._given_input_shape is not None and not self.built:
            self._ensure_built((None,) + self._given_input_shape)

    # ---- reference API -------------------------------------------------------
    def get_input_shape(self):
        return self._input_shape

    def get_output_shape(self):
        return self._output_shape

    def get_weights(self):
        """numpy arrays in Keras order (override for layout conversions)."""
        return [p.detach().float().cpu().numpy().copy() for p in self._keras_params()]

    def set_weights(self, weights):
        ps = self._keras_params()
        if len(weights) != len(ps):
            raise ValueError("%s expects %d weights, got %d" % (self.name, len(ps), len(weights)))
        with torch.no_grad():
            for p, w in zip(ps, weights):
                p.copy_(torch.as_tensor(np.asarray(w), dtype=p.dtype).reshape(p.shape))

    def get_weights_shape(self):
        return [tuple(w.shape) for w in self.get_weights()]

    def _keras_params(self):
        return [p for p in self.parameters(recurse=False)]

    def regularization_loss(self):
        r = 0.0
        for reg, pname in self._regularizers:
            p = getattr(self, pname, None)
            if p is not None and reg is not None:
                r = r + reg(p)
        return r

    def add_regularizer(self, reg, param_name):
        if reg is not None:
            self._regularizers.append((reg, param_name))

    def set_name(self, name):
        self.name = name
        return self

    def freeze(self):
        self.trainable = False
        for p in self.parameters():
            p.requires_grad_(False)
        return self

    def unfreeze(self):
        self.trainable = True
        for p in self.parameters():
            p.requires_grad_(True)
        return self

    def __repr__(self):
        return "%s(name=%s)" % (type(self).__name__, self.name)


ZooKerasLayer = Layer


class InputLayer(Layer):
    def __init__(self, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)

    def call(self, x):
        return x


def Input(shape=None, name=None):
    """Functional-API input placeholder (topology.py:409)."""
    layer = InputLayer(input_shape=shape, name=name)
    full = (None,) + to_shape(shape)
    layer._ensure_built(full)
    node = Node(layer, [], [full])
    v = node.outputs[0]
    v.name = layer.name
    return v


class Lambda(Layer):
    """Wrap an arbitrary tensor function (autograd Lambda, Lambda.scala:31-105).

    ``function`` receives torch tensors at run time; the output shape is found
    by running it once on a tiny dummy batch unless ``output_shape`` is given.
    """

    def __init__(self, function, output_shape=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.function = function
        self._fixed_out = to_shape(output_shape)

    def compute_output_shape(self, input_shape):
        if self._fixed_out is not None:
            return (None,) + self._fixed_out
        dummy = _dummy(input_shape)
        with torch.no_grad():
            out = self.function(*dummy) if isinstance(dummy, list) else self.function(dummy)
        if isinstance(out, (list, tuple)):
            return [(None,) + tuple(o.shape[1:]) for o in out]
        return (None,) + tuple(out.shape[1:])

    def call(self, x):
        return self.function(*x) if isinstance(x, list) else self.function(x)


def _dummy(shape):
    if isinstance(shape, list):
        return [_dummy(s) for s in shape]
    if getattr(shape, "no_batch", False):
        return torch.zeros(tuple(shape))
    return torch.zeros((2,) + tuple(1 if d is None else d for d in shape[1:]))
