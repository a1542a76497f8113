"""Caffe prototxt + caffemodel -> GraphNet (Zs/models/caffe/CaffeLoader.scala:63-718,
LayerConverter.scala, V1LayerConverter.scala; Net.loadCaffe).

Structure and layer parameters come from the text prototxt; weights (blobs)
from the binary NetParameter, matched by layer name. Both V2 (``layer``)
and V1 (``layers``) definitions are read. In-place layers (top == bottom,
e.g. ReLU) are chained by renaming the produced blob.

Binary schema used (caffe.proto): NetParameter 1 name, 2 layers(V1),
3 input, 4 input_dim, 8 input_shape, 100 layer; LayerParameter 1 name,
2 type, 3 bottom, 4 top, 7 blobs; V1LayerParameter 2 bottom, 3 top, 4 name,
5 type(enum), 6 blobs; BlobProto 1 num, 2 channels, 3 height, 4 width,
5 data, 7 shape(BlobShape 1 dim), 8 double_data.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo.pipeline.api.net import graph_net as G
from zoo.utils.protobuf import as_str, group, packed_doubles, packed_floats, packed_varints, parse_text

V1_TYPES = {0: "None", 35: "AbsVal", 1: "Accuracy", 30: "ArgMax", 2: "BNLL", 3: "Concat", 4: "Convolution",
            5: "Data", 39: "Deconvolution", 6: "Dropout", 25: "Eltwise", 38: "Exp", 8: "Flatten", 12: "ImageData",
            14: "InnerProduct", 15: "LRN", 29: "MemoryData", 34: "MVN", 17: "Pooling", 26: "Power", 18: "ReLU",
            19: "Sigmoid", 20: "Softmax", 21: "SoftmaxWithLoss", 22: "Split", 33: "Slice", 23: "TanH",
            31: "Threshold"}
V1_NAMES = {"CONVOLUTION": "Convolution", "INNER_PRODUCT": "InnerProduct", "POOLING": "Pooling", "RELU": "ReLU",
            "SIGMOID": "Sigmoid", "TANH": "TanH", "SOFTMAX": "Softmax", "SOFTMAX_LOSS": "SoftmaxWithLoss",
            "LRN": "LRN", "DROPOUT": "Dropout", "CONCAT": "Concat", "ELTWISE": "Eltwise", "FLATTEN": "Flatten",
            "DATA": "Data", "SPLIT": "Split", "POWER": "Power", "ABSVAL": "AbsVal", "EXP": "Exp",
            "DECONVOLUTION": "Deconvolution", "ACCURACY": "Accuracy", "BNLL": "BNLL"}


def _blob(b):
    g = group(b)
    if 5 in g:
        data = packed_floats(g[5])
    elif 8 in g:
        data = packed_doubles(g[8]).astype(np.float32)
    else:
        data = np.zeros(0, np.float32)
    if 7 in g:
        shape = packed_varints(group(g[7][0][1]).get(1, []))
    else:
        shape = [int(g[k][0][1]) if k in g else 1 for k in (1, 2, 3, 4)]
    if int(np.prod(shape)) != data.size:
        shape = [data.size]
    return data.reshape(shape)


def read_caffemodel(path):
    """layer name -> [blob arrays] (V1 and V2 layers)."""
    with open(path, "rb") as f:
        net = group(f.read())
    out = {}
    for _, lb in net.get(100, []):
        lg = group(lb)
        name = as_str(lg[1][0][1]) if 1 in lg else ""
        out[name] = [_blob(v) for _, v in lg.get(7, [])]
    for _, lb in net.get(2, []):
        lg = group(lb)
        name = as_str(lg[4][0][1]) if 4 in lg else ""
        out[name] = [_blob(v) for _, v in lg.get(6, [])]
    return out


def _p(d, key, default=None):
    v = d.get(key)
    return v[0] if v else default


def _pair(p, base, hkey, wkey, default):
    if hkey in p or wkey in p:
        return int(_p(p, hkey, default)), int(_p(p, wkey, default))
    v = p.get(base)
    if v:
        return (int(v[0]), int(v[-1]) if len(v) > 1 else int(v[0]))
    return default, default


class _InnerProduct(nn.Module):
    """Linear that flattens from ``axis`` (Caffe) and, like BigDL's converter,
    reinterprets a larger input as rows of ``in_features``."""

    def __init__(self, lin, axis=1):
        super().__init__()
        self.lin, self.axis = lin, axis

    def forward(self, x):
        x = x.flatten(self.axis)
        if x.shape[-1] != self.lin.in_features:
            x = x.reshape(-1, self.lin.in_features)
        return self.lin(x)


class _Eltwise(nn.Module):
    def __init__(self, op, coeff):
        super().__init__()
        self.op, self.coeff = op, coeff

    def forward(self, xs):
        if self.op in ("PROD", 0):
            out = xs[0]
            for t in xs[1:]:
                out = out * t
            return out
        if self.op in ("MAX", 2):
            out = xs[0]
            for t in xs[1:]:
                out = torch.maximum(out, t)
            return out
        c = self.coeff or [1.0] * len(xs)
        out = xs[0] * c[0]
        for t, k in zip(xs[1:], c[1:]):
            out = out + t * k
        return out


def _convert(ltype, p, blobs, in_channels):
    """(module, multi_input) for one Caffe layer; ``p`` is its params dict."""
    if ltype in ("Convolution", "Deconvolution"):
        cp = _p(p, "convolution_param", {})
        n_out = int(_p(cp, "num_output"))
        kh, kw = _pair(cp, "kernel_size", "kernel_h", "kernel_w", 1)
        sh, sw = _pair(cp, "stride", "stride_h", "stride_w", 1)
        ph, pw = _pair(cp, "pad", "pad_h", "pad_w", 0)
        dh, dw = _pair(cp, "dilation", "dilation_h", "dilation_w", 1)
        groups = int(_p(cp, "group", 1))
        bias = bool(_p(cp, "bias_term", True))
        w = blobs[0] if blobs else None
        if ltype == "Convolution":
            cin = w.size // (n_out * kh * kw) * groups if w is not None else in_channels
            m = nn.Conv2d(cin, n_out, (kh, kw), (sh, sw), (ph, pw), (dh, dw), groups=groups, bias=bias)
        else:
            cin = w.size // (n_out // groups * kh * kw) if w is not None else in_channels
            m = nn.ConvTranspose2d(cin, n_out, (kh, kw), (sh, sw), (ph, pw), groups=groups, bias=bias,
                                   dilation=(dh, dw))
        with torch.no_grad():
            if w is not None:
                m.weight.copy_(torch.from_numpy(w.reshape(m.weight.shape)))
            if bias and len(blobs) > 1:
                m.bias.copy_(torch.from_numpy(blobs[1].reshape(-1)))
        return m, False, n_out
    if ltype == "InnerProduct":
        ip = _p(p, "inner_product_param", {})
        n_out = int(_p(ip, "num_output"))
        bias = bool(_p(ip, "bias_term", True))
        w = blobs[0].reshape(n_out, -1) if blobs else None
        lin = nn.Linear(w.shape[1] if w is not None else in_channels, n_out, bias=bias)
        with torch.no_grad():
            if w is not None:
                lin.weight.copy_(torch.from_numpy(w))
            if bias and len(blobs) > 1:
                lin.bias.copy_(torch.from_numpy(blobs[1].reshape(-1)))
        return _InnerProduct(lin, int(_p(ip, "axis", 1))), False, n_out
    if ltype == "Pooling":
        pp = _p(p, "pooling_param", {})
        kind = "avg" if _p(pp, "pool", "MAX") in ("AVE", 1) else "max"
        kh, kw = _pair(pp, "kernel_size", "kernel_h", "kernel_w", 1)
        sh, sw = _pair(pp, "stride", "stride_h", "stride_w", 1)
        ph, pw = _pair(pp, "pad", "pad_h", "pad_w", 0)
        return G.Pool2d(kind, (kh, kw), (sh, sw), (ph, pw), ceil_mode=True,
                        global_pool=bool(_p(pp, "global_pooling", False))), False, in_channels
    if ltype == "ReLU":
        ns = float(_p(_p(p, "relu_param", {}), "negative_slope", 0.0))
        fn = torch.relu if ns == 0 else (lambda x: F.leaky_relu(x, ns))
        return G.Fn(fn, "ReLU"), False, in_channels
    if ltype in ("Sigmoid", "TanH", "AbsVal", "Exp", "BNLL"):
        fn = {"Sigmoid": torch.sigmoid, "TanH": torch.tanh, "AbsVal": torch.abs, "Exp": torch.exp,
              "BNLL": F.softplus}[ltype]
        return G.Fn(fn, ltype), False, in_channels
    if ltype in ("Softmax", "SoftmaxWithLoss"):
        axis = int(_p(_p(p, "softmax_param", {}), "axis", 1))
        return G.Fn(lambda x: F.softmax(x, dim=axis if x.dim() > axis else -1), "Softmax"), False, in_channels
    if ltype == "Dropout":
        return nn.Dropout(float(_p(_p(p, "dropout_param", {}), "dropout_ratio", 0.5))), False, in_channels
    if ltype == "LRN":
        lp = _p(p, "lrn_param", {})
        return G.LRN(int(_p(lp, "local_size", 5)), float(_p(lp, "alpha", 1.0)), float(_p(lp, "beta", 0.75)),
                     float(_p(lp, "k", 1.0))), False, in_channels
    if ltype == "Concat":
        axis = int(_p(_p(p, "concat_param", {}), "axis", 1))
        return G.JoinTable(axis), True, in_channels
    if ltype == "Eltwise":
        ep = _p(p, "eltwise_param", {})
        return _Eltwise(_p(ep, "operation", "SUM"), [float(c) for c in ep.get("coeff", [])]), True, in_channels
    if ltype == "Flatten":
        return G.Flatten(int(_p(_p(p, "flatten_param", {}), "axis", 1))), False, in_channels
    if ltype == "Reshape":
        shp = _p(_p(p, "reshape_param", {}), "shape", {})
        dims = [int(d) for d in shp.get("dim", [])]
        return G.Fn(lambda x: x.reshape([x.shape[i] if d == 0 else d for i, d in enumerate(dims)]),
                    "Reshape"), False, in_channels
    if ltype == "BatchNorm":
        bp = _p(p, "batch_norm_param", {})
        eps = float(_p(bp, "eps", 1e-5))
        mean, var = blobs[0].reshape(-1), blobs[1].reshape(-1)
        sf = float(blobs[2].reshape(-1)[0]) if len(blobs) > 2 and blobs[2].size else 1.0
        sf = 0.0 if sf == 0 else 1.0 / sf
        bn = nn.BatchNorm2d(mean.size, eps=eps, affine=False)
        with torch.no_grad():
            bn.running_mean.copy_(torch.from_numpy(mean * sf))
            bn.running_var.copy_(torch.from_numpy(var * sf))
        bn.eval()
        return bn, False, mean.size
    if ltype == "Scale":
        sp = _p(p, "scale_param", {})
        has_b = bool(_p(sp, "bias_term", False))
        return G.Scale(blobs[0].reshape(-1), blobs[1].reshape(-1) if has_b and len(blobs) > 1 else None,
                       int(_p(sp, "axis", 1))), False, in_channels
    if ltype == "Power":
        pp = _p(p, "power_param", {})
        pw_, sc, sh_ = float(_p(pp, "power", 1.0)), float(_p(pp, "scale", 1.0)), float(_p(pp, "shift", 0.0))
        return G.Fn(lambda x: (sh_ + sc * x) ** pw_, "Power"), False, in_channels
    if ltype == "PReLU":
        w = torch.from_numpy(blobs[0].reshape(-1).copy())
        m = nn.PReLU(w.numel())
        with torch.no_grad():
            m.weight.copy_(w)
        return m, False, in_channels
    if ltype in ("Split", "Silence"):
        return G.Fn(lambda x: x, ltype), False, in_channels
    raise NotImplementedError("Caffe layer type %s is not supported by the loader" % ltype)


_SKIP = ("Data", "ImageData", "MemoryData", "HDF5Data", "Accuracy", "DummyData", "Input", "WindowData")


def load_caffe(def_path, model_path=None, match_all=True):
    with open(def_path) as f:
        net = parse_text(f.read())
    blobs = read_caffemodel(model_path) if model_path else {}
    layers = net.get("layer", []) or net.get("layers", [])
    inputs = [str(x) for x in net.get("input", [])]
    dims = [int(x) for x in net.get("input_dim", [])]
    if not dims and net.get("input_shape"):
        dims = [int(x) for x in net["input_shape"][0].get("dim", [])]
    nodes = []
    producer = {}     # blob name -> node name producing its current value
    channels = {}
    for name in inputs:
        producer[name] = name
        nodes.append((name, G.NodeLayer(G.Fn(lambda x: x, "Input"), name), []))
        channels[name] = dims[1] if len(dims) > 1 else None
    for lp in layers:
        ltype = _p(lp, "type", "")
        ltype = V1_NAMES.get(ltype, ltype) if isinstance(ltype, str) else V1_TYPES.get(ltype, str(ltype))
        name = str(_p(lp, "name", ltype))
        bottoms = [str(b) for b in lp.get("bottom", [])]
        tops = [str(t) for t in lp.get("top", [])] or [name]
        if ltype in _SKIP:
            for t in tops:
                if t not in producer:
                    producer[t] = t
                    nodes.append((t, G.NodeLayer(G.Fn(lambda x: x, "Input"), t), []))
                    inputs.append(t)
                    ip = _p(lp, "input_param", {})
                    shp = _p(ip, "shape", {})
                    channels[t] = int(shp["dim"][1]) if shp and len(shp.get("dim", [])) > 1 else None
            continue
        in_nodes = [producer.get(b, b) for b in bottoms]
        cin = channels.get(bottoms[0]) if bottoms else None
        mod, multi, cout = _convert(ltype, lp, blobs.get(name, []), cin)
        if match_all and model_path and ltype in ("Convolution", "InnerProduct") and name not in blobs:
            raise ValueError("caffemodel has no weights for layer %s" % name)
        node_name = name
        if not bottoms:  # a head layer without an input: it consumes the graph input
            inputs.append(node_name)
        nodes.append((node_name, G.NodeLayer(mod, node_name, multi), in_nodes))
        for t in tops:
            producer[t] = node_name
            channels[t] = cout
    consumed = {i for _, _, ins in nodes for i in ins}
    outs = [n for n, _, _ in nodes if n not in consumed and n not in inputs] or [nodes[-1][0]]
    shape = tuple([None] + dims[1:]) if dims else None
    g = G.GraphNet(nodes, inputs, outs, name=str(_p(net, "name", "caffe")), input_shape=shape)
    g.eval()
    return g
