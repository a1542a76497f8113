"""ONNX model -> GraphNet (Py/pipeline/api/onnx/onnx_loader.py:16-128 and the 37
op mappers under Py/pipeline/api/onnx/mapper/).

The ``onnx`` package is not needed: the ModelProto is decoded with the
framework's own protobuf reader (zoo.utils.protobuf). Schema fields used:
ModelProto 7 graph, 8 opset_import; GraphProto 1 node, 2 name,
5 initializer, 11 input, 12 output; NodeProto 1 input, 2 output, 3 name,
4 op_type, 5 attribute; AttributeProto 1 name, 2 f, 3 i, 4 s, 5 t,
7 floats, 8 ints, 9 strings, 20 type; TensorProto 1 dims, 2 data_type,
4 float_data, 5 int32_data, 7 int64_data, 8 name, 9 raw_data, 10 double_data;
ValueInfoProto 1 name, 2 type (TypeProto.tensor_type.shape.dim.dim_value).
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo.pipeline.api.net import native_lower as NL

from zoo.pipeline.api.net import graph_net as G
from zoo.utils.protobuf import (as_float32, as_str, enc_bytes, enc_float, enc_int, enc_packed_ints, group,
                                packed_doubles, packed_floats, packed_varints)

_DT = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_,
       10: np.float16, 11: np.float64}


def decode_tensor(b):
    g = group(b)
    dims = packed_varints(g.get(1, []))
    dt = int(g[2][0][1]) if 2 in g else 1
    name = as_str(g[8][0][1]) if 8 in g else ""
    np_dt = _DT.get(dt, np.float32)
    if 9 in g:
        arr = np.frombuffer(g[9][0][1], dtype=np.dtype(np_dt).newbyteorder("<")).astype(np_dt)
    elif 4 in g:
        arr = packed_floats(g[4])
    elif 7 in g:
        arr = np.asarray(packed_varints(g[7]), dtype=np.int64)
    elif 5 in g:
        arr = np.asarray(packed_varints(g[5]), dtype=np_dt)
    elif 10 in g:
        arr = packed_doubles(g[10])
    else:
        arr = np.zeros(0, np_dt)
    return name, arr.reshape(dims) if dims else arr.reshape(())


def decode_attr(b):
    g = group(b)
    name = as_str(g[1][0][1])
    if 5 in g:
        return name, decode_tensor(g[5][0][1])[1]
    if 8 in g:
        return name, packed_varints(g[8])
    if 7 in g:
        return name, packed_floats(g[7]).tolist()
    if 9 in g:
        return name, [as_str(v) for _, v in g[9]]
    if 2 in g:
        w, v = g[2][0]
        return name, as_float32(w, v)
    if 3 in g:
        v = int(g[3][0][1])
        return name, v - (1 << 64) if v >= 1 << 63 else v
    if 4 in g:
        return name, as_str(g[4][0][1])
    return name, None


def _value_info(b):
    g = group(b)
    name = as_str(g[1][0][1])
    shape = []
    if 2 in g:
        tt = group(g[2][0][1])
        if 1 in tt:
            ten = group(tt[1][0][1])
            if 2 in ten:
                for _, d in group(ten[2][0][1]).get(1, []):
                    dg = group(d)
                    shape.append(int(dg[1][0][1]) if 1 in dg else None)
    return name, shape


def decode_model(data):
    m = group(data)
    gr = group(m[7][0][1])
    inits = dict(decode_tensor(v) for _, v in gr.get(5, []))
    nodes = []
    for _, nb in gr.get(1, []):
        ng = group(nb)
        nodes.append({"inputs": [as_str(v) for _, v in ng.get(1, [])],
                      "outputs": [as_str(v) for _, v in ng.get(2, [])],
                      "name": as_str(ng[3][0][1]) if 3 in ng else "",
                      "op": as_str(ng[4][0][1]),
                      "attrs": dict(decode_attr(v) for _, v in ng.get(5, []))})
    inputs = [_value_info(v) for _, v in gr.get(11, [])]
    outputs = [_value_info(v)[0] for _, v in gr.get(12, [])]
    return {"nodes": nodes, "inits": inits, "inputs": [(n, s) for n, s in inputs if n not in inits],
            "outputs": outputs, "name": as_str(gr[2][0][1]) if 2 in gr else "onnx"}


# ---- op mappers -----------------------------------------------------------------------------
class OnnxOp(nn.Module):
    """Generic node: constant inputs become parameters/buffers, the runtime
    inputs arrive as a list in ONNX input order."""

    def __init__(self, op, attrs, const_inputs, n_inputs):
        super().__init__()
        self.op, self.attrs, self.n_inputs = op, attrs, n_inputs
        self.const_slots = {}
        self.params = nn.ParameterDict()
        for slot, (name, arr) in const_inputs.items():
            key = "c%d" % slot
            t = torch.from_numpy(np.ascontiguousarray(arr))
            if t.is_floating_point():
                self.params[key] = nn.Parameter(t.float(), requires_grad=op in _TRAINABLE)
            else:
                self.register_buffer(key, t)
            self.const_slots[slot] = key

    def _gather_inputs(self, xs):
        out, it = [], iter(xs)
        for slot in range(self.n_inputs):
            if slot in self.const_slots:
                k = self.const_slots[slot]
                out.append(self.params[k] if k in self.params else getattr(self, k))
            else:
                out.append(next(it, None))
        return out

    def forward(self, xs):
        xs = xs if isinstance(xs, list) else [xs]
        return _OPS[self.op](self._gather_inputs(xs), self.attrs)


_TRAINABLE = {"Conv", "Gemm", "MatMul", "BatchNormalization", "ConvTranspose", "PRelu"}


def _pads(a, nd=2):
    p = a.get("pads", [0] * (2 * nd))
    return p


def _conv(x, a):
    inp, w = x[0], x[1]
    b = x[2] if len(x) > 2 else None
    p = _pads(a)
    if a.get("auto_pad", "NOTSET") in ("SAME_UPPER", "SAME_LOWER"):
        return _same_conv(inp, w, b, a)
    if p[0] != p[2] or p[1] != p[3]:
        inp = F.pad(inp, (p[1], p[3], p[0], p[2]))
        p = [0, 0, 0, 0]
    y = NL.conv2d_nchw(inp, w, b, tuple(a.get("strides", [1, 1])), (p[0], p[1]), tuple(a.get("dilations", [1, 1])),
                       a.get("group", 1))
    if y is not None:   # the native implicit-GEMM kernels (GPU, groups == 1)
        return y
    return F.conv2d(inp, w, b, tuple(a.get("strides", [1, 1])), (p[0], p[1]), tuple(a.get("dilations", [1, 1])),
                    a.get("group", 1))


def _same_conv(inp, w, b, a):
    s = a.get("strides", [1, 1])
    k = w.shape[-2:]
    ih, iw = inp.shape[-2:]
    oh, ow = -(-ih // s[0]), -(-iw // s[1])
    ph, pw = max((oh - 1) * s[0] + k[0] - ih, 0), max((ow - 1) * s[1] + k[1] - iw, 0)
    inp = F.pad(inp, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
    y = NL.conv2d_nchw(inp, w, b, tuple(s), (0, 0), tuple(a.get("dilations", [1, 1])), a.get("group", 1))
    if y is not None:
        return y
    return F.conv2d(inp, w, b, tuple(s), 0, tuple(a.get("dilations", [1, 1])), a.get("group", 1))


def _gemm(x, a):
    A, B = x[0], x[1]
    if (A.is_cuda and A.dim() == 2 and B.dim() == 2 and not a.get("transA", 0) and a.get("alpha", 1.0) == 1.0 and
            (len(x) < 3 or x[2] is None or (a.get("beta", 1.0) == 1.0 and x[2].dim() == 1))):
        # Y = A B^T (+ c): the native MFMA linear with the bias in its epilogue
        W = B if a.get("transB", 0) else B.t()
        from zoo import ops
        return ops.linear(A, W, x[2] if len(x) > 2 else None)
    if a.get("transA", 0):
        A = A.t()
    if a.get("transB", 0):
        B = B.t()
    y = a.get("alpha", 1.0) * (A @ B)
    if len(x) > 2 and x[2] is not None:
        y = y + a.get("beta", 1.0) * x[2]
    return y


def _pool(kind):
    def f(x, a):
        k = a["kernel_shape"]
        s = a.get("strides", [1] * len(k))
        p = _pads(a)
        inp = x[0]
        if p[0] != p[2] or p[1] != p[3]:
            inp = F.pad(inp, (p[1], p[3], p[0], p[2]), value=float("-inf") if kind == "max" else 0.0)
            p = [0, 0, 0, 0]
        if inp.dim() == 4 and len(k) == 2:
            y = NL.pool2d_nchw(inp, kind, tuple(k), tuple(s), (p[0], p[1]), bool(a.get("ceil_mode", 0)),
                               bool(a.get("count_include_pad", 0)))
            if y is not None:
                return y
        if kind == "max":
            return F.max_pool2d(inp, k, s, (p[0], p[1]), ceil_mode=bool(a.get("ceil_mode", 0)))
        return F.avg_pool2d(inp, k, s, (p[0], p[1]), ceil_mode=bool(a.get("ceil_mode", 0)),
                            count_include_pad=bool(a.get("count_include_pad", 0)))
    return f


def _bn(x, a):
    if x[0].dim() == 4:
        y = NL.batch_norm_nchw_eval(x[0], x[3], x[4], x[1], x[2], a.get("epsilon", 1e-5))
        if y is not None:
            return y
    return F.batch_norm(x[0], x[3], x[4], x[1], x[2], False, 0.0, a.get("epsilon", 1e-5))


def _reshape(x, a):
    shape = [int(v) for v in (x[1].tolist() if len(x) > 1 else a["shape"])]
    shape = [x[0].shape[i] if v == 0 else v for i, v in enumerate(shape)]
    return x[0].reshape(shape)


def _softmax(fn):
    def f(x, a):
        axis = a.get("axis", -1)
        return fn(x[0], dim=axis)
    return f


def _flatten(x, a):
    axis = a.get("axis", 1)
    return x[0].reshape(int(np.prod(x[0].shape[:axis])) if axis else 1, -1)


def _unsqueeze(x, a):
    axes = a.get("axes") or x[1].tolist()
    y = x[0]
    for ax in sorted(axes):
        y = y.unsqueeze(ax)
    return y


def _squeeze(x, a):
    axes = a.get("axes") or (x[1].tolist() if len(x) > 1 and x[1] is not None else None)
    if not axes:
        return x[0].squeeze()
    y = x[0]
    for ax in sorted(axes, reverse=True):
        y = y.squeeze(ax)
    return y


def _reduce(fn):
    def f(x, a):
        axes = a.get("axes") or (x[1].tolist() if len(x) > 1 and x[1] is not None else None)
        keep = bool(a.get("keepdims", 1))
        if axes is None:
            return fn(x[0]) if not keep else fn(x[0]).reshape([1] * x[0].dim())
        return fn(x[0], dim=tuple(axes), keepdim=keep)
    return f


def _clip(x, a):
    lo = x[1] if len(x) > 1 and x[1] is not None else a.get("min", -3.4e38)
    hi = x[2] if len(x) > 2 and x[2] is not None else a.get("max", 3.4e38)
    return torch.clamp(x[0], float(lo), float(hi))


def _pad(x, a):
    pads = a.get("pads") or x[1].tolist()
    n = len(pads) // 2
    tp = []
    for i in reversed(range(n)):
        tp += [pads[i], pads[i + n]]
    return F.pad(x[0], tp, mode={"constant": "constant", "reflect": "reflect", "edge": "replicate"}[
        a.get("mode", "constant")])


def _many(fn):
    def f(x, a):
        out = x[0]
        for t in x[1:]:
            out = fn(out, t)
        return out
    return f


def _act(x, name, ref):
    y = NL.activation(x, name)
    return ref(x) if y is None else y


def _gap(x):
    y = NL.global_avg_pool_nchw(x) if x.dim() == 4 else None
    return x.mean(dim=tuple(range(2, x.dim())), keepdim=True) if y is None else y


_OPS = {
    "Conv": _conv, "Gemm": _gemm, "MatMul": lambda x, a: x[0] @ x[1],
    "Add": lambda x, a: x[0] + x[1], "Sub": lambda x, a: x[0] - x[1], "Mul": lambda x, a: x[0] * x[1],
    "Div": lambda x, a: x[0] / x[1], "Pow": lambda x, a: x[0] ** x[1], "Neg": lambda x, a: -x[0],
    "Relu": lambda x, a: _act(x[0], "relu", torch.relu), "Sigmoid": lambda x, a: _act(x[0], "sigmoid", torch.sigmoid),
    "Tanh": lambda x, a: _act(x[0], "tanh", torch.tanh), "Exp": lambda x, a: torch.exp(x[0]), "Log": lambda x, a: torch.log(x[0]),
    "Sqrt": lambda x, a: torch.sqrt(x[0]), "Abs": lambda x, a: torch.abs(x[0]),
    "Erf": lambda x, a: torch.erf(x[0]), "Softsign": lambda x, a: F.softsign(x[0]),
    "Softplus": lambda x, a: F.softplus(x[0]),
    "LeakyRelu": lambda x, a: F.leaky_relu(x[0], a.get("alpha", 0.01)),
    "Elu": lambda x, a: F.elu(x[0], a.get("alpha", 1.0)),
    "HardSigmoid": lambda x, a: torch.clamp(a.get("alpha", 0.2) * x[0] + a.get("beta", 0.5), 0, 1),
    "PRelu": lambda x, a: torch.where(x[0] >= 0, x[0], x[0] * x[1]),
    "Softmax": _softmax(F.softmax), "LogSoftmax": _softmax(F.log_softmax),
    "MaxPool": _pool("max"), "AveragePool": _pool("avg"),
    "GlobalAveragePool": lambda x, a: _gap(x[0]),
    "GlobalMaxPool": lambda x, a: x[0].amax(dim=tuple(range(2, x[0].dim())), keepdim=True),
    "BatchNormalization": _bn, "Flatten": _flatten, "Reshape": _reshape,
    "Transpose": lambda x, a: x[0].permute(a.get("perm") or list(reversed(range(x[0].dim())))),
    "Concat": lambda x, a: torch.cat([t for t in x if t is not None], a.get("axis", 0)),
    "Dropout": lambda x, a: x[0], "Identity": lambda x, a: x[0],
    "Unsqueeze": _unsqueeze, "Squeeze": _squeeze, "Clip": _clip, "Pad": _pad,
    "ReduceMean": _reduce(torch.mean), "ReduceSum": _reduce(torch.sum),
    "ReduceMax": _reduce(lambda t, dim=None, keepdim=False: t.amax(dim=dim, keepdim=keepdim) if dim is not None
                         else t.max()),
    "Sum": _many(torch.add), "Max": _many(torch.maximum), "Min": _many(torch.minimum),
    "Mean": lambda x, a: sum(x) / len(x),
    "Gather": lambda x, a: torch.index_select(x[0], a.get("axis", 0), x[1].reshape(-1).long()).reshape(
        tuple(x[0].shape[:a.get("axis", 0)]) + tuple(x[1].shape) + tuple(x[0].shape[a.get("axis", 0) + 1:])),
    "Shape": lambda x, a: torch.tensor(list(x[0].shape), dtype=torch.int64),
    "Cast": lambda x, a: x[0].float() if a.get("to", 1) == 1 else x[0].long() if a.get("to") == 7 else x[0],
    "LRN": lambda x, a: F.local_response_norm(x[0], a["size"], a.get("alpha", 1e-4), a.get("beta", 0.75),
                                              a.get("bias", 1.0)),
    "Upsample": lambda x, a: F.interpolate(x[0], scale_factor=tuple(x[1].tolist()[2:]) if len(x) > 1 else
                                           tuple(a["scales"][2:]), mode="nearest"),
    "ConvTranspose": lambda x, a: F.conv_transpose2d(x[0], x[1], x[2] if len(x) > 2 else None,
                                                     tuple(a.get("strides", [1, 1])), tuple(_pads(a)[:2]),
                                                     groups=a.get("group", 1)),
}


def supported_ops():
    return sorted(_OPS)


def graph_from_model(model):
    inits = model["inits"]
    nodes = []
    produced = {}
    const_values = dict(inits)
    for i, nd in enumerate(model["nodes"]):
        op = nd["op"]
        name = nd["name"] or "%s_%d" % (op, i)
        if op == "Constant":
            const_values[nd["outputs"][0]] = nd["attrs"].get("value")
            continue
        if op not in _OPS:
            raise NotImplementedError("ONNX op %s is not supported (supported: %s)" % (op, ", ".join(supported_ops())))
        consts = {s: (n, const_values[n]) for s, n in enumerate(nd["inputs"]) if n in const_values}
        runtime = [n for n in nd["inputs"] if n and n not in const_values]
        mod = OnnxOp(op, nd["attrs"], consts, len(nd["inputs"]))
        ins = [produced.get(n, n) for n in runtime]
        nodes.append((name, G.NodeLayer(mod, name, multi_input=True), ins))
        for o in nd["outputs"]:
            produced[o] = name
    in_names = [n for n, _ in model["inputs"]]
    src = [(n, G.NodeLayer(G.Fn(lambda x: x, "Input"), n), []) for n in in_names]
    outs = [produced.get(o, o) for o in model["outputs"]]
    shape = model["inputs"][0][1] if model["inputs"] else None
    g = G.GraphNet(src + nodes, in_names, outs, name=model["name"],
                   input_shape=tuple([None] + list(shape[1:])) if shape else None)
    g.eval()
    return g


def load_onnx(path):
    with open(path, "rb") as f:
        return graph_from_model(decode_model(f.read()))


class OnnxLoader:
    """Py/pipeline/api/onnx/onnx_loader.py OnnxLoader facade."""

    def __init__(self, path):
        self.path = path

    @staticmethod
    def from_path(path, is_training=False):
        return load_onnx(path)

    def to_keras(self):
        return load_onnx(self.path)


# ---- writer (builds ONNX files for tests / export of simple graphs) ---------------------------
def enc_tensor(name, arr):
    arr = np.asarray(arr)
    dt = {np.dtype(np.float32): 1, np.dtype(np.int64): 7, np.dtype(np.int32): 6}[arr.dtype]
    return enc_packed_ints(1, arr.shape) + enc_int(2, dt) + enc_bytes(8, name) + enc_bytes(9, arr.tobytes())


def enc_attr(name, v):
    out = enc_bytes(1, name)
    if isinstance(v, float):
        return out + enc_float(2, v) + enc_int(20, 1)
    if isinstance(v, int):
        return out + enc_int(3, v) + enc_int(20, 2)
    if isinstance(v, str):
        return out + enc_bytes(4, v) + enc_int(20, 3)
    if isinstance(v, (list, tuple)):
        return out + enc_packed_ints(8, v) + enc_int(20, 7)
    raise TypeError(v)


def enc_node(op, inputs, outputs, name="", **attrs):
    out = b"".join(enc_bytes(1, i) for i in inputs) + b"".join(enc_bytes(2, o) for o in outputs)
    out += enc_bytes(3, name) + enc_bytes(4, op)
    for k, v in attrs.items():
        out += enc_bytes(5, enc_attr(k, v))
    return out


def enc_value_info(name, shape):
    dims = b"".join(enc_bytes(1, enc_int(1, d)) for d in shape)
    tensor = enc_int(1, 1) + enc_bytes(2, dims)
    return enc_bytes(1, name) + enc_bytes(2, enc_bytes(1, tensor))


def make_model(nodes, inputs, outputs, initializers, name="g"):
    gr = b"".join(enc_bytes(1, n) for n in nodes) + enc_bytes(2, name)
    gr += b"".join(enc_bytes(5, enc_tensor(k, v)) for k, v in initializers.items())
    gr += b"".join(enc_bytes(11, enc_value_info(n, s)) for n, s in inputs)
    gr += b"".join(enc_bytes(12, enc_value_info(n, s)) for n, s in outputs)
    return enc_int(1, 7) + enc_bytes(7, gr) + enc_bytes(8, enc_bytes(1, "") + enc_int(2, 13))
