"""GraphNet: an imported DAG of modules (BigDL StaticGraph / Caffe net /
ONNX graph) behind the Keras model API.

Reference: Zs/pipeline/api/net/NetUtils.scala:47-140 (GraphNet with
``newGraph(outputs)``, ``freezeUpTo``, ``node(name)``), Python
Py/pipeline/api/net/graph_net.py. Each graph node becomes a Keras ``Layer``
(so ``layers``, ``flattened_layers``, ``get_layer``, freeze/unfreeze and
compile/fit/predict all work); the graph is evaluated in topological order.
Imported models keep their source layout (NCHW) at the API; ``to_native()`` (done by the
Net loaders on GPU, by InferenceModel and by Cluster Serving) swaps every supported node for a
native twin running the zoo NHWC kernels (``native_lower.py``), with channels-last tensors
flowing between native nodes.
"""
import numpy as np
import torch
import torch.nn as nn

from zoo.pipeline.api.keras.base import Layer
from zoo.pipeline.api.keras.engine.topology import KerasNet


class NodeLayer(Layer):
    """Wraps one imported op (an nn.Module taking a tensor or a list)."""

    def __init__(self, module, name, multi_input=False):
        super().__init__(name=name)
        self.op = module
        self.multi_input = multi_input
        self.built = True

    def call(self, x):
        return self.op(x)

    def compute_output_shape(self, input_shape):
        return None

    def _keras_params(self):
        return list(self.op.parameters())


class GraphNet(KerasNet):
    def __init__(self, nodes, inputs, outputs, name=None, input_shape=None):
        """nodes: ordered list of (name, NodeLayer, [input names]); inputs: graph
        input names (fed positionally); outputs: names of the result nodes."""
        super().__init__(name=name)
        self.node_names = [n for n, _, _ in nodes]
        self.node_inputs = {n: list(i) for n, _, i in nodes}
        self.nodes = nn.ModuleDict()
        for n, layer, _ in nodes:
            self.nodes[_key(n)] = layer
        self.inputs = list(inputs)
        self.outputs = list(outputs)
        self._input_shape = input_shape
        self.built = True
        self._order = self._toposort()

    def _toposort(self):
        needed = set()
        stack = list(self.outputs)
        while stack:
            n = stack.pop()
            if n in needed or n in self.inputs and n not in self.node_inputs:
                continue
            needed.add(n)
            stack.extend(self.node_inputs.get(n, []))
        order, done = [], set(self.inputs) - set(self.node_inputs)
        pending = [n for n in self.node_names if n in needed]
        while pending:
            progressed = False
            for n in list(pending):
                if all(i in done for i in self.node_inputs[n]):
                    order.append(n)
                    done.add(n)
                    pending.remove(n)
                    progressed = True
            if not progressed:
                raise ValueError("graph has a cycle or a missing input: %s" % pending)
        return order

    def node(self, name):
        return self.nodes[_key(name)]

    def to_native(self, training=False):
        """Run this imported graph on the native NHWC kernels (zoo.pipeline.api.net.native_lower):
        every conv / linear / pooling / batch-norm / activation / LRN / LSTM node gets a native
        twin sharing its parameters; in inference, conv -> BN -> activation chains fuse into one
        kernel. In place; returns self."""
        from zoo.pipeline.api.net.native_lower import lower_graph
        return lower_graph(self, training)

    def _layer_list(self):
        return [self.nodes[_key(n)] for n in self.node_names]

    def compute_output_shape(self, input_shape):
        return self._output_shape

    def call(self, x):
        xs = x if isinstance(x, (list, tuple)) else [x]
        vals = {}
        for name, t in zip(self.inputs, xs):
            vals[name] = t
        for n in self._order:
            ins = self.node_inputs[n]
            layer = self.nodes[_key(n)]
            if not ins:  # a source node consumes the next graph input
                arg = vals[n] if n in vals else xs[self.inputs.index(n)] if n in self.inputs else xs[0]
            elif layer.multi_input:
                arg = [vals[i] for i in ins]
            else:
                arg = vals[ins[0]]
            vals[n] = layer.op(arg)
        outs = [vals[o] for o in self.outputs]
        return outs[0] if len(outs) == 1 else outs

    def forward(self, x, *rest):
        if rest:
            x = [x] + list(rest)
        return self.call(x)

    def new_graph(self, outputs):
        """A graph sharing these layers whose outputs are ``outputs`` (NetUtils.newGraph)."""
        outputs = [outputs] if isinstance(outputs, str) else list(outputs)
        nodes = [(n, self.nodes[_key(n)], self.node_inputs[n]) for n in self.node_names]
        g = GraphNet(nodes, self.inputs, outputs, name=self.name + "_sub", input_shape=self._input_shape)
        keep = set(g._order)
        g.node_names = [n for n in self.node_names if n in keep]
        g.nodes = nn.ModuleDict({_key(n): self.nodes[_key(n)] for n in g.node_names})
        return g

    def _ancestors(self, names):
        out, stack = set(), list(names)
        while stack:
            n = stack.pop()
            if n in out:
                continue
            out.add(n)
            stack.extend(self.node_inputs.get(n, []))
        return out

    def freeze_up_to(self, names):
        """Freeze every node that feeds (or is) one of ``names`` (NetUtils.freezeUpTo)."""
        names = [names] if isinstance(names, str) else list(names)
        for n in self._ancestors(names):
            if _key(n) in self.nodes:
                self.nodes[_key(n)].freeze()
        return self

    def unfreeze(self, names=None):
        for n in self.node_names:
            if names is None or n in names:
                self.nodes[_key(n)].unfreeze()
        return self

    @torch.no_grad()
    def forward_numpy(self, x):
        was = self.training
        self.eval()
        xs = [torch.as_tensor(np.asarray(t), dtype=torch.float32) for t in (x if isinstance(x, list) else [x])]
        dev = next(iter(self.parameters()), torch.zeros(0)).device
        out = self.call([t.to(dev) for t in xs] if len(xs) > 1 else xs[0].to(dev))
        self.train(was)
        return out.cpu().numpy() if torch.is_tensor(out) else [o.cpu().numpy() for o in out]

    def predict_numpy(self, x):
        return self.forward_numpy(x)


def _key(name):
    return name.replace(".", "_")


# ---- shared op modules (NCHW) ---------------------------------------------------------------
class Reshape(nn.Module):
    """BigDL Reshape(size, batchMode): batch dim kept unless the input is exactly ``size``."""

    def __init__(self, size, batch_mode=None):
        super().__init__()
        self.size = list(size)
        self.batch_mode = batch_mode

    def forward(self, x):
        n = int(np.prod(self.size))
        if self.batch_mode is False or (self.batch_mode is None and x.dim() == len(self.size)
                                        and x.numel() == n):
            return x.reshape(self.size)
        return x.reshape([x.shape[0]] + self.size)


class View(Reshape):
    pass


class Flatten(nn.Module):
    def __init__(self, axis=1):
        super().__init__()
        self.axis = axis

    def forward(self, x):
        return x.flatten(self.axis)


class Fn(nn.Module):
    def __init__(self, fn, name=""):
        super().__init__()
        self.fn = fn
        self.fname = name

    def forward(self, x):
        return self.fn(x)

    def extra_repr(self):
        return self.fname


class CAddTable(nn.Module):
    def forward(self, xs):
        out = xs[0]
        for t in xs[1:]:
            out = out + t
        return out


class CMulTable(nn.Module):
    def forward(self, xs):
        out = xs[0]
        for t in xs[1:]:
            out = out * t
        return out


class CMaxTable(nn.Module):
    def forward(self, xs):
        out = xs[0]
        for t in xs[1:]:
            out = torch.maximum(out, t)
        return out


class JoinTable(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, xs):
        return torch.cat(xs, self.dim)


class Scale(nn.Module):
    """Per-channel affine (Caffe Scale / BigDL CMul+CAdd on dim 1)."""

    def __init__(self, weight, bias=None, axis=1):
        super().__init__()
        self.weight = nn.Parameter(torch.as_tensor(weight, dtype=torch.float32))
        self.bias = None if bias is None else nn.Parameter(torch.as_tensor(bias, dtype=torch.float32))
        self.axis = axis

    def forward(self, x):
        shape = [1] * x.dim()
        shape[self.axis] = -1
        y = x * self.weight.reshape(shape)
        return y + self.bias.reshape(shape) if self.bias is not None else y


class Pool2d(nn.Module):
    def __init__(self, kind, kernel, stride, pad, ceil_mode=False, global_pool=False, count_include_pad=True):
        super().__init__()
        self.kind, self.kernel, self.stride, self.pad = kind, kernel, stride, pad
        self.ceil_mode, self.global_pool, self.count_include_pad = ceil_mode, global_pool, count_include_pad

    def forward(self, x):
        import torch.nn.functional as F
        k = tuple(x.shape[-2:]) if self.global_pool else self.kernel
        s = k if self.global_pool else self.stride
        p = (0, 0) if self.global_pool else self.pad
        if self.kind == "max":
            return F.max_pool2d(x, k, s, p, ceil_mode=self.ceil_mode)
        return F.avg_pool2d(x, k, s, p, ceil_mode=self.ceil_mode, count_include_pad=self.count_include_pad)


class LRN(nn.Module):
    def __init__(self, size, alpha, beta, k):
        super().__init__()
        self.size, self.alpha, self.beta, self.k = size, alpha, beta, k

    def forward(self, x):
        import torch.nn.functional as F
        return F.local_response_norm(x, self.size, self.alpha, self.beta, self.k)
