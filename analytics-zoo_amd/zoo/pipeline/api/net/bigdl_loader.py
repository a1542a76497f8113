"""BigDL ``.model`` -> GraphNet (Net.loadBigDL, Zs/pipeline/api/Net.scala:110-140;
module registry K11, Topology.scala:708-825).

Supports the module types BigDL models are built from (graph containers
StaticGraph / Sequential / Concat / ConcatTable, Linear, SpatialConvolution,
SpatialMaxPooling / SpatialAveragePooling, (Spatial)BatchNormalization,
activations, Reshape / View, tables, Dropout, LogSoftMax / SoftMax, ...).
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo.pipeline.api.net import graph_net as G
from zoo.utils.bigdl_proto import TensorRef, load_bigdl_spec


def _t(ref, storages):
    return None if ref is None else torch.from_numpy(ref.materialize(storages).copy())


def _attr(spec, k, default=None):
    v = spec.attr.get(k, default)
    return default if v is None else v


def _conv(spec, st):
    a = spec.attr
    n_in, n_out, g = a["nInputPlane"], a["nOutputPlane"], a.get("nGroup", 1) or 1
    kw, kh = a["kernelW"], a["kernelH"]
    sw, sh = a.get("strideW", 1), a.get("strideH", 1)
    pw, ph = a.get("padW", 0), a.get("padH", 0)
    same = pw == -1 or ph == -1
    dil = (int(a.get("dilationH", 1) or 1), int(a.get("dilationW", 1) or 1))
    conv = nn.Conv2d(n_in, n_out, (kh, kw), (sh, sw), 0 if same else (ph, pw), dilation=dil, groups=g,
                     bias=spec.bias is not None and a.get("withBias", True) is not False)
    with torch.no_grad():
        conv.weight.copy_(_t(spec.weight, st).reshape(conv.weight.shape))
        if conv.bias is not None:
            conv.bias.copy_(_t(spec.bias, st).reshape(-1))
    if not same:
        return conv

    class Same(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = conv

        def forward(self, x):
            ih, iw = x.shape[-2:]
            oh, ow = -(-ih // sh), -(-iw // sw)
            ph_ = max((oh - 1) * sh + kh - ih, 0)
            pw_ = max((ow - 1) * sw + kw - iw, 0)
            x = F.pad(x, (pw_ // 2, pw_ - pw_ // 2, ph_ // 2, ph_ - ph_ // 2))
            return self.conv(x)
    return Same()


def _linear(spec, st):
    a = spec.attr
    lin = nn.Linear(a["inputSize"], a["outputSize"], bias=spec.bias is not None)
    with torch.no_grad():
        lin.weight.copy_(_t(spec.weight, st).reshape(lin.weight.shape))
        if lin.bias is not None:
            lin.bias.copy_(_t(spec.bias, st).reshape(-1))
    return lin


def _bn(spec, st, spatial):
    a = spec.attr
    n = a.get("nOutput") or (spec.weight.size[0] if spec.weight else None)
    bn = (nn.BatchNorm2d if spatial else nn.BatchNorm1d)(n, eps=float(a.get("eps", 1e-5)),
                                                         momentum=float(a.get("momentum", 0.1)),
                                                         affine=spec.weight is not None)
    with torch.no_grad():
        if spec.weight is not None:
            bn.weight.copy_(_t(spec.weight, st).reshape(-1))
            bn.bias.copy_(_t(spec.bias, st).reshape(-1))
        for key, buf in (("runningMean", bn.running_mean), ("runningVar", bn.running_var)):
            v = a.get(key)
            if isinstance(v, TensorRef):
                buf.copy_(torch.from_numpy(v.materialize(st)).reshape(-1))
    return bn


def _pool(spec, kind):
    a = spec.attr
    return G.Pool2d(kind, (a["kH"], a["kW"]), (a.get("dH", 1), a.get("dW", 1)), (a.get("padH", 0), a.get("padW", 0)),
                    ceil_mode=bool(a.get("ceil_mode", a.get("ceilMode", False))),
                    global_pool=bool(a.get("globalPooling", False)),
                    count_include_pad=bool(a.get("countIncludePad", True)))


def _batch_mode(v):
    if isinstance(v, bool):
        return v
    return {1: True, 2: False}.get(v)


def _lsm(x):
    from zoo.ops.nn import softmax
    return softmax(x, -1, log=True)


def _sm(x):
    from zoo.ops.nn import softmax
    return softmax(x, -1)


def convert(spec, st):
    """BigDLModuleSpec -> (nn.Module, multi_input)."""
    t = spec.short_type
    a = spec.attr
    if t == "Linear":
        return _linear(spec, st), False
    if t in ("SpatialConvolution", "SpatialShareConvolution", "SpatialDilatedConvolution"):
        return _conv(spec, st), False
    if t == "SpatialMaxPooling":
        return _pool(spec, "max"), False
    if t == "SpatialAveragePooling":
        return _pool(spec, "avg"), False
    if t == "SpatialBatchNormalization":
        return _bn(spec, st, True), False
    if t == "BatchNormalization":
        return _bn(spec, st, False), False
    if t in ("Reshape", "InferReshape"):
        return G.Reshape(a.get("size", []), _batch_mode(a.get("batchMode"))), False
    if t == "View":
        return G.View(a.get("sizes", a.get("size", [])), None), False
    if t in ("Tanh", "ReLU", "Sigmoid", "Identity", "LogSoftMax", "SoftMax", "ReLU6", "SoftPlus", "SoftSign",
             "Abs", "Exp", "Log", "Sqrt", "Square", "HardTanh"):
        fn = {"Tanh": torch.tanh, "ReLU": torch.relu, "Sigmoid": torch.sigmoid, "Identity": lambda x: x,
              "LogSoftMax": _lsm, "SoftMax": _sm, "ReLU6": lambda x: F.relu6(x), "SoftPlus": F.softplus,
              "SoftSign": F.softsign, "Abs": torch.abs, "Exp": torch.exp, "Log": torch.log, "Sqrt": torch.sqrt,
              "Square": torch.square, "HardTanh": lambda x: torch.clamp(x, -1, 1)}[t]
        return G.Fn(fn, t), False
    if t == "Input":
        return G.Fn(lambda x: x, t), False
    if t == "Narrow":
        d, off, ln = int(a.get("dimension", 1)), int(a.get("offset", 1)), int(a.get("length", 1))
        return G.Fn(lambda x: x.narrow(d - 1, off - 1, ln if ln > 0 else x.shape[d - 1] - off + 2 + ln), t), False
    if t == "LeakyReLU":
        ns = float(a.get("negval", 0.01))
        return G.Fn(lambda x: F.leaky_relu(x, ns), t), False
    if t == "Dropout":
        return nn.Dropout(float(a.get("initP", 0.5))), False
    if t == "CAddTable":
        return G.CAddTable(), True
    if t == "CMulTable":
        return G.CMulTable(), True
    if t == "CMaxTable":
        return G.CMaxTable(), True
    if t == "JoinTable":
        dim = int(a.get("dimension", 2))
        n_in = int(a.get("nInputDims", 0) or 0)
        return G.JoinTable(dim - 1 if n_in == 0 else dim), True  # 1-based dim; batch offset when nInputDims set
    if t == "SpatialCrossMapLRN":
        return G.LRN(int(a.get("size", 5)), float(a.get("alpha", 1e-4)), float(a.get("beta", 0.75)),
                     float(a.get("k", 1.0))), False
    if t in ("Sequential", "StaticGraph", "Graph", "DynamicGraph", "Model"):
        return build_graph(spec, st), False
    raise NotImplementedError("BigDL module type %s (%s) is not supported by the loader" % (spec.type, spec.name))


def _edges(spec, node):
    e = spec.attr.get(node.name + "_edges")
    if isinstance(e, dict):
        return list(e["attr"].keys())
    return list(node.pre)


def build_graph(spec, st):
    t = spec.short_type
    if t == "Sequential":
        nodes, prev = [], None
        for sub in spec.submodules:
            mod, multi = convert(sub, st)
            nodes.append((sub.name, G.NodeLayer(mod, sub.name, multi), [] if prev is None else [prev]))
            prev = sub.name
        first = nodes[0][0] if nodes else "input"
        return G.GraphNet(nodes, [first], [prev], name=spec.name)
    nodes = []
    for sub in spec.submodules:
        mod, multi = convert(sub, st)
        nodes.append((sub.name, G.NodeLayer(mod, sub.name, multi), _edges(spec, sub)))
    ins = spec.attr.get("inputNames")
    outs = spec.attr.get("outputNames")
    ins = ins if isinstance(ins, list) and ins else [n for n, _, i in nodes if not i]
    outs = outs if isinstance(outs, list) and outs else [nodes[0][0]]
    # the file lists nodes outputs-first; keep a stable inputs-first order
    shape = None
    first = next((s for s in spec.submodules if s.name == ins[0]), None) if ins else None
    if first is not None and first.short_type == "Reshape" and first.attr.get("size"):
        shape = (None,) + tuple(first.attr["size"])
    return G.GraphNet(list(reversed(nodes)), ins, outs, name=spec.name, input_shape=shape)


def load_bigdl(path, weight_path=None):
    spec, storages = load_bigdl_spec(path)
    if weight_path is not None:
        _, wst = load_bigdl_spec(weight_path)
        storages.update(wst)
    g = build_graph(spec, storages) if spec.submodules else G.GraphNet(
        [(spec.name, G.NodeLayer(convert(spec, storages)[0], spec.name), [])], [spec.name], [spec.name])
    g.eval()
    return g
