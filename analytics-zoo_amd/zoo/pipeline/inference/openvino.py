"""OpenVINO IR (``.xml`` topology + ``.bin`` weights) loader and executor.

The reference hands IR files to Intel's OpenVINO CPU runtime through JNI
(``Zs/pipeline/inference/OpenVINOModel.scala:40-130``,
``OpenVinoInferenceSupportive.scala``; Python ``InferenceModel.load_openvino``,
``pyzoo/zoo/pipeline/inference/inference_model.py:69-79``). There is no such runtime
for MI355X, so the IR is decoded here and executed by this framework:

* IR v10/v11 (opset graphs: ``Parameter``/``Const``/op layers + ``<edges>``) and the
  legacy IR v5-v7 (``Input`` + layers whose weights sit in ``<blobs>``) are parsed with
  the standard-library XML reader; weights are read from the ``.bin`` blob by
  (offset, size, element type) with numpy (no code in the files is executed).
* The graph becomes an ``nn.Module`` whose layers run in topological order. On the GPU
  the compute-heavy layers take the native kernels: ``Convolution`` (groups == 1) runs
  the implicit-GEMM MFMA conv on a channels-last view (weights packed once),
  ``MatMul``/``FullyConnected`` run ``zoo.ops.linear``, ``MaxPool`` the native NHWC
  pooling kernel; everything else is a PyTorch op on the same tensors.
* ``FakeQuantize`` (the int8 IRs of ``OpenVINOInt8Suite.scala``) is evaluated
  numerically, so calibrated int8 IRs produce the quantised network's outputs.

Unsupported layer types raise ``NotImplementedError`` naming the type and layer.
"""
import math
import xml.etree.ElementTree as ET

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

_NP_TYPES = {"f32": np.float32, "fp32": np.float32, "f16": np.float16, "fp16": np.float16, "f64": np.float64,
             "i64": np.int64, "i32": np.int32, "i8": np.int8, "u8": np.uint8, "i16": np.int16, "u16": np.uint16,
             "boolean": np.bool_, "u1": np.uint8, "bf16": None}
_TORCH_TYPES = {"f32": torch.float32, "f16": torch.float16, "f64": torch.float64, "i64": torch.int64,
                "i32": torch.int32, "i8": torch.int8, "u8": torch.uint8, "boolean": torch.bool,
                "bf16": torch.bfloat16}


def _ints(s, default=None):
    if s is None or s == "":
        return default
    return [int(v) for v in str(s).split(",") if v.strip() != ""]


def _floats(s):
    return [float(v) for v in str(s).split(",") if v.strip() != ""]


def _port_dims(port):
    return [int(d.text) for d in port.findall("dim")]


class _Layer:
    __slots__ = ("id", "name", "type", "attrs", "inputs", "out_ports", "const", "version", "blobs", "precision",
                 "out_dims")

    def __init__(self, el):
        self.id = el.get("id")
        self.name = el.get("name", self.id)
        self.type = el.get("type")
        self.version = el.get("version", "")
        self.precision = el.get("precision", "FP32")
        d = el.find("data")
        self.attrs = dict(d.attrib) if d is not None else {}
        self.inputs = []          # [(from_layer_id, from_port)] ordered by input port id
        outs = el.find("output")
        self.out_ports = [p.get("id") for p in outs.findall("port")] if outs is not None else []
        self.out_dims = {p.get("id"): _port_dims(p) for p in outs.findall("port")} if outs is not None else {}
        self.const = None
        self.blobs = {}
        b = el.find("blobs")
        if b is not None:
            for c in b:
                self.blobs[c.tag] = (int(c.get("offset")), int(c.get("size")), c.get("precision"))


def _read_blob(bin_bytes, offset, size, etype, shape=None):
    if etype == "bf16":
        raw = np.frombuffer(bin_bytes, dtype=np.uint16, count=size // 2, offset=offset)
        t = torch.from_numpy(raw.astype(np.int32) << 16).view(torch.float32)
        return t.reshape(shape) if shape else t
    dt = _NP_TYPES.get(etype)
    if dt is None:
        raise NotImplementedError("OpenVINO IR: element type %r" % etype)
    n = size // np.dtype(dt).itemsize
    a = np.frombuffer(bin_bytes, dtype=dt, count=n, offset=offset).copy()
    if shape is not None and len(shape):
        a = a.reshape(shape)
    elif shape is not None:
        a = a.reshape(())
    t = torch.from_numpy(a)
    return t.float() if t.dtype == torch.float16 else t


class OpenVINOModel(nn.Module):
    """An IR graph executed by this framework. ``forward(*inputs)`` takes the
    ``Parameter`` inputs in IR order and returns the ``Result`` tensor(s)."""

    def __init__(self, xml_path, bin_path=None, batch_size=0):
        super().__init__()
        root = ET.parse(xml_path).getroot()
        self.ir_version = int(root.get("version", "10"))
        self.batch_size = int(batch_size or 0)
        blob = b""
        if bin_path is not None:
            with open(bin_path, "rb") as f:
                blob = f.read()
        layers = {}
        order = []
        for el in root.find("layers"):
            L = _Layer(el)
            layers[L.id] = L
            order.append(L.id)
        ins = {}
        for e in root.find("edges"):
            ins.setdefault(e.get("to-layer"), []).append((int(e.get("to-port")), e.get("from-layer"),
                                                         e.get("from-port")))
        for lid, lst in ins.items():
            layers[lid].inputs = [(fl, fp) for _, fl, fp in sorted(lst)]
        self._consts = {}
        for lid in order:
            L = layers[lid]
            if L.type == "Const":
                a = L.attrs
                shape = _ints(a.get("shape"), [])
                et = a.get("element_type") or {"FP32": "f32", "FP16": "f16", "I64": "i64",
                                                "I32": "i32"}.get(L.precision, "f32")
                if "offset" not in a:  # legacy Const with a custom blob
                    off, size, prec = L.blobs["custom"]
                    et = {"FP32": "f32", "FP16": "f16", "I64": "i64", "I32": "i32"}.get(prec or L.precision, "f32")
                    shape = L.out_dims[L.out_ports[0]]
                else:
                    off, size = int(a["offset"]), int(a["size"])
                t = _read_blob(blob, off, size, et, shape)
                self._consts[lid] = t
            elif L.blobs:
                prec = {"FP32": "f32", "FP16": "f16"}.get(L.precision, "f32")
                for k, (off, size, p) in L.blobs.items():
                    pe = {"FP32": "f32", "FP16": "f16", "I64": "i64", "I32": "i32"}.get(p, prec)
                    L.blobs[k] = _read_blob(blob, off, size, pe)
        # register float constants as buffers so .to(device) moves them
        self._buf_names = {}
        for i, (lid, t) in enumerate(self._consts.items()):
            name = "c%d" % i
            self.register_buffer(name, t, persistent=False)
            self._buf_names[lid] = name
        for lid in order:
            L = layers[lid]
            if isinstance(L.blobs, dict):
                for k, v in list(L.blobs.items()):
                    if isinstance(v, torch.Tensor):
                        name = "b_%s_%s" % (lid, k)
                        self.register_buffer(name, v, persistent=False)
                        L.blobs[k] = name
        self.layers = layers
        self.order = self._toposort(order, layers)
        self.inputs = [lid for lid in order if layers[lid].type in ("Parameter", "Input")]
        self.outputs = [lid for lid in order if layers[lid].type == "Result"]
        if not self.outputs:  # legacy IR: layers nobody consumes are the outputs
            used = {fl for L in layers.values() for fl, _ in L.inputs}
            self.outputs = [lid for lid in order if lid not in used and layers[lid].type not in ("Const",)]
        self._native_w = {}
        self.input_names = [layers[i].name for i in self.inputs]

    @staticmethod
    def _toposort(order, layers):
        seen, out = set(), []

        def visit(lid):
            if lid in seen:
                return
            seen.add(lid)
            for fl, _ in layers[lid].inputs:
                visit(fl)
            out.append(lid)
        for lid in order:
            visit(lid)
        return out

    # ------------------------------------------------------------------ helpers
    def _blob(self, L, key):
        v = L.blobs.get(key)
        return None if v is None else getattr(self, v)

    def _conv(self, L, x, w, b, strides, pads_b, pads_e, dil, groups):
        nd = w.dim() - 2
        if list(pads_b) != list(pads_e):   # asymmetric padding: pad explicitly, convolve unpadded
            pad = []
            for i in reversed(range(nd)):
                pad += [pads_b[i], pads_e[i]]
            x = F.pad(x, pad)
            pads = (0,) * nd
        else:
            pads = tuple(pads_b)
        if x.is_cuda and groups == 1 and nd == 2:
            return self._conv_native(L, x, w, b, strides, pads, dil)
        xf = x.float() if x.dtype != w.dtype else x
        fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[nd]
        return fn(xf, w.to(xf.dtype), None if b is None else b.to(xf.dtype).reshape(-1), tuple(strides), pads,
                  tuple(dil), groups)

    def _conv_native(self, L, x, w, b, strides, pads, dil):
        from zoo import ops
        K, C, R, S = w.shape
        cin_p = C if C % 8 == 0 else (4 if C <= 4 else ops.ceil8(C))
        k_p = ops.ceil8(K)
        key = L.id
        cached = self._native_w.get(key)
        if cached is None or cached[0].device != x.device:
            w4 = torch.zeros(k_p, R, S, cin_p, device=x.device)
            w4[:K, :, :, :C] = w.float().permute(0, 2, 3, 1)
            bp = None
            if b is not None:
                bp = torch.zeros(k_p, device=x.device)
                bp[:K] = b.float().reshape(-1)
            cached = (ops.pack_weight(w4), bp)
            self._native_w[key] = cached
        xn = x.permute(0, 2, 3, 1)
        if cin_p != C:
            xn = F.pad(xn, (0, cin_p - C))
        y = ops.conv2d_nhwc(xn.to(torch.bfloat16).contiguous(), cached[0], cached[1], kernel=(R, S),
                            stride=tuple(strides), pad=list(pads), dil=tuple(dil), out_f32=True)
        return y[..., :K].permute(0, 3, 1, 2)

    @staticmethod
    def _auto_pads(L, x, kernel, strides, dil):
        a = L.attrs
        ap = a.get("auto_pad", "explicit")
        pb = _ints(a.get("pads_begin"), [0] * len(kernel))
        pe = _ints(a.get("pads_end"), [0] * len(kernel))
        if ap in ("same_upper", "same_lower"):
            pb, pe = [], []
            for i, k in enumerate(kernel):
                n = x.shape[2 + i]
                eff = dil[i] * (k - 1) + 1
                out = int(math.ceil(n / strides[i]))
                tot = max((out - 1) * strides[i] + eff - n, 0)
                lo = tot // 2 if ap == "same_upper" else tot - tot // 2
                pb.append(lo)
                pe.append(tot - lo)
        elif ap == "valid":
            pb, pe = [0] * len(kernel), [0] * len(kernel)
        return pb, pe

    def _pool(self, L, x, kind, kernel, strides, pb, pe, ceil, exclude_pad=True):
        if any(p != q for p, q in zip(pb, pe)):
            pad = []
            for i in reversed(range(len(kernel))):
                pad += [pb[i], pe[i]]
            x = F.pad(x, pad, value=float("-inf") if kind == "max" else 0.0)
            pb = [0] * len(kernel)
        if kind == "max":
            if x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0:
                from zoo import ops
                y = ops.max_pool2d_nhwc(x.permute(0, 2, 3, 1), tuple(kernel), tuple(strides), tuple(pb),
                                        ceil_mode=ceil)
                return y.permute(0, 3, 1, 2).to(x.dtype)
            fn = F.max_pool2d if x.dim() == 4 else (F.max_pool1d if x.dim() == 3 else F.max_pool3d)
            return fn(x, tuple(kernel), tuple(strides), tuple(pb), ceil_mode=ceil)
        fn = F.avg_pool2d if x.dim() == 4 else (F.avg_pool1d if x.dim() == 3 else F.avg_pool3d)
        return fn(x, tuple(kernel), tuple(strides), tuple(pb), ceil_mode=ceil, count_include_pad=not exclude_pad)

    # ------------------------------------------------------------------ forward
    def forward(self, *inputs):
        vals = {}
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = tuple(inputs[0])
        if len(inputs) != len(self.inputs):
            raise ValueError("OpenVINO model expects %d inputs, got %d" % (len(self.inputs), len(inputs)))
        for lid, t in zip(self.inputs, inputs):
            t = torch.as_tensor(t)
            et = self.layers[lid].attrs.get("element_type", "f32")
            if t.is_floating_point() and et in ("f32", "f16"):
                t = t.float()
            vals[(lid, self.layers[lid].out_ports[0] if self.layers[lid].out_ports else "0")] = t
        for lid in self.order:
            L = self.layers[lid]
            if L.type in ("Parameter", "Input"):
                continue
            if L.type == "Const":
                vals[(lid, L.out_ports[0])] = getattr(self, self._buf_names[lid])
                continue
            args = [vals[(fl, fp)] for fl, fp in L.inputs]
            out = self._run(L, args)
            if not isinstance(out, (list, tuple)):
                out = [out]
            for port, v in zip(L.out_ports or ["0"], out):
                vals[(lid, port)] = v
            if L.type == "Result":
                vals[(lid, "result")] = out[0]
        res = []
        for lid in self.outputs:
            L = self.layers[lid]
            res.append(vals[(lid, "result")] if L.type == "Result" else vals[(lid, (L.out_ports or ["0"])[0])])
        return res[0] if len(res) == 1 else res

    def predict(self, inputs):
        with torch.no_grad():
            return self.forward(inputs)

    # ------------------------------------------------------------------ ops
    def _run(self, L, a):  # noqa: C901 - one dispatch table
        t, at = L.type, L.attrs
        if t == "Result":
            return a[0]
        if t == "Convolution":
            if len(a) > 1:                  # v10: weights are an input [K, C, k...]
                w, b, groups = a[1], None, 1
            else:                           # legacy: weights in blobs, [K, C/g, kh, kw] flattened
                groups = int(at.get("group", 1))
                kernel = _ints(at.get("kernel") or ",".join([at.get("kernel-y"), at.get("kernel-x")]))
                K = int(at.get("output"))
                w = self._blob(L, "weights").reshape(K, a[0].shape[1] // groups, *kernel)
                b = self._blob(L, "biases")
            kernel = list(w.shape[2:])
            strides = _ints(at.get("strides"), [1] * len(kernel))
            dil = _ints(at.get("dilations"), [1] * len(kernel))
            pb, pe = self._auto_pads(L, a[0], kernel, strides, dil)
            return self._conv(L, a[0], w, b, strides, pb, pe, dil, groups)
        if t == "GroupConvolution":
            w = a[1]
            G = w.shape[0]
            w = w.reshape(G * w.shape[1], *w.shape[2:])
            kernel = list(w.shape[2:])
            strides = _ints(at.get("strides"), [1] * len(kernel))
            dil = _ints(at.get("dilations"), [1] * len(kernel))
            pb, pe = self._auto_pads(L, a[0], kernel, strides, dil)
            return self._conv(L, a[0], w, None, strides, pb, pe, dil, G)
        if t in ("MaxPool", "AvgPool", "Pooling"):
            kernel = _ints(at.get("kernel"))
            strides = _ints(at.get("strides"), [1] * len(kernel))
            pb, pe = self._auto_pads(L, a[0], kernel, strides, [1] * len(kernel))
            ceil = at.get("rounding_type", "floor") == "ceil"
            kind = "max" if t == "MaxPool" or at.get("pool-method", "max") == "max" else "avg"
            excl = str(at.get("exclude-pad", "true")).lower() == "true"
            y = self._pool(L, a[0], kind, kernel, strides, pb, pe, ceil, excl)
            return [y, torch.zeros_like(y, dtype=torch.int64)] if len(L.out_ports) > 1 else y
        if t == "MatMul":
            x, w = a
            if at.get("transpose_a", "false") == "true":
                x = x.transpose(-1, -2)
            tb = at.get("transpose_b", "false") == "true"
            if x.is_cuda and w.dim() == 2 and x.dim() >= 2 and x.is_floating_point():
                from zoo import ops
                wt = w if tb else w.t()
                return ops.linear(x.float(), wt.float().contiguous())
            return torch.matmul(x, w.transpose(-1, -2) if tb else w)
        if t == "FullyConnected":
            K = int(at.get("out-size"))
            x = a[0].reshape(a[0].shape[0], -1)
            w = self._blob(L, "weights").reshape(K, -1)
            b = self._blob(L, "biases")
            if x.is_cuda:
                from zoo import ops
                return ops.linear(x.float(), w.float(), None if b is None else b.float())
            return F.linear(x, w, b)
        if t in ("Add", "Subtract", "Multiply", "Divide", "Maximum", "Minimum", "Power", "SquaredDifference",
                 "Equal", "Less", "Greater", "LogicalAnd"):
            x, y = a
            if x.is_floating_point() != y.is_floating_point():
                y = y.to(x.dtype) if x.is_floating_point() else y
                x = x.to(y.dtype) if y.is_floating_point() else x
            return {"Add": torch.add, "Subtract": torch.sub, "Multiply": torch.mul,
                    "Divide": (lambda p, q: torch.div(p, q, rounding_mode="floor") if not p.is_floating_point()
                               else p / q),
                    "Maximum": torch.maximum, "Minimum": torch.minimum, "Power": torch.pow,
                    "SquaredDifference": lambda p, q: (p - q) ** 2, "Equal": torch.eq, "Less": torch.lt,
                    "Greater": torch.gt, "LogicalAnd": torch.logical_and}[t](x, y)
        if t == "Eltwise":
            op = at.get("operation", "sum").lower()
            out = a[0]
            coeff = _floats(at["coeff"]) if at.get("coeff") else None
            for i, v in enumerate(a[1:], 1):
                if op in ("sum", "add"):
                    out = out * (coeff[0] if coeff and i == 1 else 1.0) + v * (coeff[i] if coeff else 1.0)
                elif op in ("mul", "prod"):
                    out = out * v
                elif op == "max":
                    out = torch.maximum(out, v)
                elif op == "sub":
                    out = out - v
                else:
                    raise NotImplementedError("OpenVINO IR: Eltwise operation %r (layer %s)" % (op, L.name))
            return out
        if t == "ScaleShift":
            w = self._blob(L, "weights")
            b = self._blob(L, "biases")
            shp = [1, -1] + [1] * (a[0].dim() - 2)
            y = a[0] * w.reshape(shp) if w is not None else a[0]
            return y + b.reshape(shp) if b is not None else y
        if t in ("Relu", "ReLU"):
            slope = float(at.get("negative_slope", 0))
            return F.leaky_relu(a[0], slope) if slope else torch.relu(a[0])
        if t == "PReLU" or t == "PRelu":
            s = a[1] if len(a) > 1 else self._blob(L, "weights")
            if s.numel() > 1 and a[0].dim() > 2:
                s = s.reshape([1, -1] + [1] * (a[0].dim() - 2))
            return torch.where(a[0] >= 0, a[0], a[0] * s)
        if t == "Clamp":
            return torch.clamp(a[0], float(at.get("min")), float(at.get("max")))
        if t == "Elu":
            return F.elu(a[0], float(at.get("alpha", 1.0)))
        if t in ("Gelu",):
            return F.gelu(a[0], approximate="tanh" if at.get("approximation_mode", "erf").lower() == "tanh"
                          else "none")
        if t == "Activation":
            kind = at.get("type", "").lower()
            return {"sigmoid": torch.sigmoid, "tanh": torch.tanh, "relu": torch.relu, "elu": F.elu}[kind](a[0])
        unary = {"Sigmoid": torch.sigmoid, "Tanh": torch.tanh, "Exp": torch.exp, "Log": torch.log,
                 "Sqrt": torch.sqrt, "Abs": torch.abs, "Negative": torch.neg, "Floor": torch.floor,
                 "Ceiling": torch.ceil, "Erf": torch.erf, "HSwish": F.hardswish, "HSigmoid": F.hardsigmoid,
                 "Mish": F.mish, "SoftPlus": F.softplus, "Sin": torch.sin, "Cos": torch.cos,
                 "LogicalNot": torch.logical_not}
        if t in unary:
            return unary[t](a[0])
        if t == "Swish":
            beta = a[1] if len(a) > 1 else 1.0
            return a[0] * torch.sigmoid(a[0] * beta)
        if t == "Power" and not a[1:]:  # legacy Power: (shift + scale * x) ^ power
            return (float(at.get("shift", 0)) + float(at.get("scale", 1)) * a[0]) ** float(at.get("power", 1))
        if t in ("SoftMax", "Softmax", "LogSoftmax"):
            axis = int(at.get("axis", 1))
            return F.log_softmax(a[0], axis) if t == "LogSoftmax" else torch.softmax(a[0], axis)
        if t == "BatchNormInference":
            x, g, b, m, v = a
            eps = float(at.get("epsilon", 1e-5))
            shp = [1, -1] + [1] * (x.dim() - 2)
            return (x - m.reshape(shp)) / torch.sqrt(v.reshape(shp) + eps) * g.reshape(shp) + b.reshape(shp)
        if t == "BatchNormalization":  # legacy: scale/shift blobs hold the folded BN
            return self._run(_Proxy(L, "ScaleShift"), a)
        if t in ("Reshape",):
            if len(a) > 1:
                shape = [int(v) for v in a[1].reshape(-1).tolist()]
                if at.get("special_zero", "false") == "true":
                    shape = [a[0].shape[i] if s == 0 else s for i, s in enumerate(shape)]
            else:
                shape = _ints(at.get("dim"))
                shape = [a[0].shape[i] if s == 0 else s for i, s in enumerate(shape)]
            return a[0].reshape(shape)
        if t == "Flatten":
            axis = int(at.get("axis", 1))
            return a[0].reshape(*a[0].shape[:axis], -1)
        if t in ("Transpose", "Permute"):
            perm = [int(v) for v in a[1].reshape(-1).tolist()] if len(a) > 1 else _ints(at.get("order"))
            return a[0].permute(perm)
        if t == "Concat":
            axis = int(at.get("axis", 1))
            if not a[0].is_floating_point() and any(v.is_floating_point() for v in a):
                a = [v.float() for v in a]
            return torch.cat(a, axis)
        if t in ("Squeeze", "Unsqueeze"):
            axes = sorted(int(v) for v in a[1].reshape(-1).tolist()) if len(a) > 1 else _ints(at.get("dim"))
            x = a[0]
            if t == "Squeeze":
                if not axes:
                    return x.squeeze()
                for ax in sorted((ax % x.dim() for ax in axes), reverse=True):
                    x = x.squeeze(ax)
                return x
            for ax in axes:
                x = x.unsqueeze(ax if ax >= 0 else ax + x.dim() + 1)
            return x
        if t in ("ReduceMean", "ReduceSum", "ReduceMax", "ReduceMin", "ReduceProd", "ReduceL2"):
            axes = [int(v) for v in a[1].reshape(-1).tolist()]
            keep = at.get("keep_dims", "false") == "true"
            x = a[0]
            if t == "ReduceMean":
                return x.mean(axes, keepdim=keep)
            if t == "ReduceSum":
                return x.sum(axes, keepdim=keep)
            if t == "ReduceL2":
                return torch.sqrt((x * x).sum(axes, keepdim=keep))
            if t == "ReduceMax":
                return torch.amax(x, axes, keepdim=keep)
            if t == "ReduceMin":
                return torch.amin(x, axes, keepdim=keep)
            out = x
            for ax in sorted((ax % x.dim() for ax in axes), reverse=True):
                out = out.prod(ax, keepdim=keep)
            return out
        if t == "ShapeOf":
            return torch.tensor(list(a[0].shape), dtype=torch.int64, device=a[0].device)
        if t == "Convert":
            return a[0].to(_TORCH_TYPES.get(at.get("destination_type", "f32"), torch.float32))
        if t == "Gather":
            axis = int(a[2].reshape(-1)[0].item()) if len(a) > 2 else int(at.get("axis", 0))
            idx = a[1].long()
            x = a[0]
            axis = axis % x.dim()
            idx = torch.where(idx < 0, idx + x.shape[axis], idx)
            out = torch.index_select(x, axis, idx.reshape(-1))
            return out.reshape(*x.shape[:axis], *idx.shape, *x.shape[axis + 1:])
        if t == "StridedSlice":
            x = a[0]
            begin = a[1].reshape(-1).tolist()
            end = a[2].reshape(-1).tolist()
            stride = a[3].reshape(-1).tolist() if len(a) > 3 else [1] * len(begin)
            bm = _ints(at.get("begin_mask"), [0] * len(begin))
            em = _ints(at.get("end_mask"), [0] * len(begin))
            sl = []
            for i in range(len(begin)):
                b_ = None if (i < len(bm) and bm[i]) else int(begin[i])
                e_ = None if (i < len(em) and em[i]) else int(end[i])
                sl.append(slice(b_, e_, int(stride[i])))
            return x[tuple(sl)]
        if t == "Split" or t == "VariadicSplit":
            axis = int(a[1].reshape(-1)[0].item())
            if t == "Split":
                return list(torch.chunk(a[0], int(at.get("num_splits")), axis))
            sizes = [int(v) for v in a[2].reshape(-1).tolist()]
            if -1 in sizes:
                i = sizes.index(-1)
                sizes[i] = a[0].shape[axis] - (sum(sizes) + 1)
            return list(torch.split(a[0], sizes, axis))
        if t == "Pad":
            pb = [int(v) for v in a[1].reshape(-1).tolist()]
            pe = [int(v) for v in a[2].reshape(-1).tolist()]
            val = float(a[3].reshape(-1)[0].item()) if len(a) > 3 else 0.0
            pad = []
            for i in reversed(range(len(pb))):
                pad += [pb[i], pe[i]]
            mode = at.get("pad_mode", "constant")
            return F.pad(a[0], pad, mode="constant" if mode == "constant" else
                         {"reflect": "reflect", "edge": "replicate"}[mode], value=val if mode == "constant" else None)
        if t == "Tile":
            return a[0].repeat([int(v) for v in a[1].reshape(-1).tolist()])
        if t == "Broadcast":
            return a[0].expand([int(v) for v in a[1].reshape(-1).tolist()])
        if t == "FakeQuantize":
            x, il, ih, ol, oh = a
            levels = float(at.get("levels", 256))
            xc = torch.minimum(torch.maximum(x, il), ih)
            q = torch.round((xc - il) / (ih - il) * (levels - 1))
            return q / (levels - 1) * (oh - ol) + ol
        if t == "NormalizeL2":
            axes = [int(v) for v in a[1].reshape(-1).tolist()]
            eps = float(at.get("eps", 1e-10))
            n = (a[0] * a[0]).sum(axes, keepdim=True)
            n = n + eps if at.get("eps_mode", "add") == "add" else torch.clamp(n, min=eps)
            return a[0] / torch.sqrt(n)
        if t == "MVN":
            x = a[0]
            axes = [int(v) for v in a[1].reshape(-1).tolist()] if len(a) > 1 else \
                (list(range(1, x.dim())) if at.get("across_channels", "false") == "true" else list(range(2, x.dim())))
            eps = float(at.get("eps", 1e-9))
            m = x.mean(axes, keepdim=True)
            y = x - m
            if at.get("normalize_variance", "true") == "true":
                v = (y * y).mean(axes, keepdim=True)
                y = y / (torch.sqrt(v + eps) if at.get("eps_mode", "inside_sqrt") == "inside_sqrt"
                         else torch.sqrt(v) + eps)
            return y
        if t == "Interpolate":
            x = a[0]
            mode = at.get("mode", "nearest")
            shape_calc = at.get("shape_calculation_mode", "sizes")
            if shape_calc == "scales" and len(a) > 2:
                scales = a[2].reshape(-1).tolist()
                size = [int(math.floor(x.shape[2 + i] * scales[-(x.dim() - 2) + i])) for i in range(x.dim() - 2)]
            else:
                sz = [int(v) for v in a[1].reshape(-1).tolist()]
                size = sz[-(x.dim() - 2):]
            m = {"nearest": "nearest", "linear": "bilinear", "linear_onnx": "bilinear", "cubic": "bicubic"}[mode]
            kw = {} if m == "nearest" else {"align_corners": at.get("coordinate_transformation_mode") ==
                                                              "align_corners"}
            return F.interpolate(x, size=size, mode=m, **kw)
        if t == "Range":
            return torch.arange(a[0].item(), a[1].item(), a[2].item(), device=a[0].device)
        if t == "Select":
            return torch.where(a[0].bool(), a[1], a[2])
        if t == "TopK":
            k = int(a[1].reshape(-1)[0].item())
            v, i = torch.topk(a[0], k, int(at.get("axis", -1)), largest=at.get("mode", "max") == "max")
            return [v, i]
        if t == "Crop":
            axes = _ints(at.get("axis"))
            offs = _ints(at.get("offset"))
            dims = _ints(at.get("dim"))
            x = a[0]
            for ax, o, d in zip(axes, offs, dims):
                x = x.narrow(ax, o, d)
            return x
        raise NotImplementedError("OpenVINO IR: layer type %r (layer %r) is not supported" % (t, L.name))


class _Proxy:
    def __init__(self, L, t):
        self.__dict__.update({k: getattr(L, k) for k in _Layer.__slots__})
        self.type = t


def load_openvino(xml_path, bin_path=None, batch_size=0):
    """Parse an OpenVINO IR into an executable :class:`OpenVINOModel`."""
    if bin_path is None:
        import os
        cand = os.path.splitext(xml_path)[0] + ".bin"
        bin_path = cand if os.path.exists(cand) else None
    return OpenVINOModel(xml_path, bin_path, batch_size).eval()


__all__ = ["OpenVINOModel", "load_openvino"]
