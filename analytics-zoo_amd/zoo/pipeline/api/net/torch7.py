"""Torch7 ``.t7`` model files (Net.loadTorch, Zs/pipeline/api/Net.scala; BigDL's TorchFile
reader). The Lua Torch binary serialisation is decoded here (no Lua, nothing executed)
and the ``nn`` container / layer objects are rebuilt as PyTorch modules:

* objects: nil / number (double) / string / boolean / table / torch class instances
  (version string ``V <n>`` + class name + payload), back-references by object index;
* tensors: dims, sizes, strides, 1-based storage offset, then the storage object
  (``torch.<Type>Storage``: element count + raw data); 8-byte longs by default;
* modules: nn.Sequential / Concat / ConcatTable / Parallel-free tables, Linear,
  SpatialConvolution(MM), SpatialMaxPooling / AveragePooling, (Spatial)BatchNormalization,
  ReLU / Threshold / Tanh / Sigmoid / SoftMax / LogSoftMax / Dropout / Identity / View /
  Reshape / CAddTable / JoinTable.

``write_t7`` (a writer for the same format) exists for tests and for exporting.
"""
import struct

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

NIL, NUMBER, STRING, TABLE, TORCH, BOOLEAN, FUNCTION, LEGACY_RECUR, RECUR = 0, 1, 2, 3, 4, 5, 6, 7, 8
_STORAGE = {"torch.FloatStorage": np.float32, "torch.DoubleStorage": np.float64, "torch.LongStorage": np.int64,
            "torch.IntStorage": np.int32, "torch.ByteStorage": np.uint8, "torch.CharStorage": np.int8,
            "torch.ShortStorage": np.int16, "torch.HalfStorage": np.float16,
            "torch.CudaStorage": np.float32, "torch.CudaDoubleStorage": np.float64}
_TENSORS = {k.replace("Storage", "Tensor"): v for k, v in _STORAGE.items()}


class T7Object:
    """A torch class instance that is not a tensor / storage: ``cls`` + ``fields``."""

    def __init__(self, cls, fields):
        self.cls, self.fields = cls, fields

    def __getitem__(self, k):
        return self.fields[k]

    def get(self, k, d=None):
        return self.fields.get(k, d) if isinstance(self.fields, dict) else d

    def __repr__(self):
        return "T7Object(%s)" % self.cls


class _Reader:
    def __init__(self, buf, long_size=8):
        self.b, self.p, self.long = buf, 0, long_size
        self.objects = {}

    def int(self):
        v = struct.unpack_from("<i", self.b, self.p)[0]
        self.p += 4
        return v

    def long_(self):
        v = struct.unpack_from("<q" if self.long == 8 else "<i", self.b, self.p)[0]
        self.p += self.long
        return v

    def double(self):
        v = struct.unpack_from("<d", self.b, self.p)[0]
        self.p += 8
        return v

    def string(self):
        n = self.int()
        s = self.b[self.p:self.p + n]
        self.p += n
        return s.decode("latin-1")

    def obj(self):
        t = self.int()
        if t == NIL:
            return None
        if t == NUMBER:
            return self.double()
        if t == STRING:
            return self.string()
        if t == BOOLEAN:
            return self.int() == 1
        if t in (TABLE, TORCH, FUNCTION, RECUR, LEGACY_RECUR):
            idx = self.int()
            if idx in self.objects:
                return self.objects[idx]
            if t == TORCH:
                ver = self.string()
                cls = self.string() if ver.startswith("V ") else ver
                if cls in _STORAGE:
                    n = self.long_()
                    dt = np.dtype(_STORAGE[cls])
                    a = np.frombuffer(self.b, dt, count=n, offset=self.p).copy()
                    self.p += n * dt.itemsize
                    self.objects[idx] = a
                    return a
                if cls in _TENSORS:
                    nd = self.int()
                    sizes = [self.long_() for _ in range(nd)]
                    strides = [self.long_() for _ in range(nd)]
                    off = self.long_() - 1
                    holder = {}
                    self.objects[idx] = holder
                    st = self.obj()
                    if st is None or nd == 0:
                        arr = np.zeros([0], _TENSORS[cls])
                    else:
                        item = st.itemsize
                        arr = np.lib.stride_tricks.as_strided(st[off:], shape=sizes,
                                                              strides=[s * item for s in strides]).copy()
                    self.objects[idx] = arr
                    return arr
                o = T7Object(cls, None)
                self.objects[idx] = o
                o.fields = self.obj()
                return o
            if t == TABLE:
                n = self.int()
                d = {}
                self.objects[idx] = d
                for _ in range(n):
                    k = self.obj()
                    d[k] = self.obj()
                return d
            # functions: dumped bytecode + upvalues; kept opaque
            size = self.int()
            self.p += size
            up = self.obj()
            return T7Object("function", up)
        raise ValueError("Torch7 file: unknown object type %d at byte %d" % (t, self.p - 4))


def read_t7(path, long_size=8):
    with open(path, "rb") as f:
        return _Reader(f.read(), long_size).obj()


def _as_list(tbl):
    if isinstance(tbl, dict):
        keys = sorted(k for k in tbl if isinstance(k, float))
        return [tbl[k] for k in keys]
    return list(tbl or [])


# ---------------------------------------------------------------------------
# nn modules
# ---------------------------------------------------------------------------
class _View(nn.Module):
    def __init__(self, size, num_input_dims=None):
        super().__init__()
        self.size = [int(s) for s in size]

    def forward(self, x):
        n = int(np.prod([s for s in self.size if s > 0]))
        if x.numel() == n:
            return x.reshape(self.size)
        return x.reshape([x.shape[0]] + self.size)


class _ConcatTable(nn.Module):
    def __init__(self, mods):
        super().__init__()
        self.mods = nn.ModuleList(mods)

    def forward(self, x):
        return [m(x) for m in self.mods]


class _Concat(nn.Module):
    def __init__(self, mods, dim):
        super().__init__()
        self.mods, self.dim = nn.ModuleList(mods), dim

    def forward(self, x):
        d = self.dim if x.dim() > 1 and self.dim < x.dim() else self.dim - 1
        return torch.cat([m(x) for m in self.mods], d)


class _CAdd(nn.Module):
    def forward(self, xs):
        out = xs[0]
        for x in xs[1:]:
            out = out + x
        return out


class _Join(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, xs):
        return torch.cat(list(xs), self.dim)


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


def to_module(o):  # noqa: C901 - one table
    """T7Object (an nn module) -> torch.nn.Module."""
    cls = o.cls.split(".")[-1] if isinstance(o, T7Object) else None
    f = o.fields if isinstance(o, T7Object) else {}
    g = lambda k, d=None: f.get(k, d)  # noqa: E731
    if cls == "Sequential":
        return nn.Sequential(*[to_module(m) for m in _as_list(g("modules"))])
    if cls == "Concat":
        return _Concat([to_module(m) for m in _as_list(g("modules"))], int(g("dimension", 2)) - 1)
    if cls == "ConcatTable":
        return _ConcatTable([to_module(m) for m in _as_list(g("modules"))])
    if cls == "CAddTable":
        return _CAdd()
    if cls == "JoinTable":
        return _Join(int(g("dimension", 2)) - 1)
    if cls == "Linear":
        w = g("weight")
        m = nn.Linear(w.shape[1], w.shape[0], bias=g("bias") is not None)
        with torch.no_grad():
            m.weight.copy_(_t(w))
            if g("bias") is not None:
                m.bias.copy_(_t(g("bias")))
        return m
    if cls in ("SpatialConvolution", "SpatialConvolutionMM"):
        cin, cout = int(g("nInputPlane")), int(g("nOutputPlane"))
        kh, kw = int(g("kH")), int(g("kW"))
        m = nn.Conv2d(cin, cout, (kh, kw), (int(g("dH", 1)), int(g("dW", 1))),
                      (int(g("padH", 0)), int(g("padW", 0))), bias=g("bias") is not None)
        with torch.no_grad():
            m.weight.copy_(_t(g("weight")).reshape(cout, cin, kh, kw))
            if g("bias") is not None:
                m.bias.copy_(_t(g("bias")))
        return m
    if cls in ("SpatialMaxPooling", "SpatialAveragePooling"):
        k = (int(g("kH")), int(g("kW")))
        s = (int(g("dH", k[0])), int(g("dW", k[1])))
        p = (int(g("padH", 0)), int(g("padW", 0)))
        ceil = bool(g("ceil_mode", False))
        if cls == "SpatialMaxPooling":
            return nn.MaxPool2d(k, s, p, ceil_mode=ceil)
        return nn.AvgPool2d(k, s, p, ceil_mode=ceil, count_include_pad=bool(g("count_include_pad", True)))
    if cls in ("SpatialBatchNormalization", "BatchNormalization"):
        rm = g("running_mean")
        n = len(rm)
        aff = g("weight") is not None
        m = (nn.BatchNorm2d if cls.startswith("Spatial") else nn.BatchNorm1d)(n, eps=float(g("eps", 1e-5)),
                                                                               momentum=float(g("momentum", 0.1)),
                                                                               affine=aff)
        with torch.no_grad():
            m.running_mean.copy_(_t(rm))
            m.running_var.copy_(_t(g("running_var")))
            if aff:
                m.weight.copy_(_t(g("weight")))
                m.bias.copy_(_t(g("bias")))
        return m
    if cls == "ReLU":
        return nn.ReLU()
    if cls == "Threshold":
        th, val = float(g("threshold", 0)), float(g("val", 0))
        return nn.Threshold(th, val)
    if cls == "Tanh":
        return nn.Tanh()
    if cls == "Sigmoid":
        return nn.Sigmoid()
    if cls == "SoftMax":
        return nn.Softmax(dim=-1)
    if cls == "LogSoftMax":
        return nn.LogSoftmax(dim=-1)
    if cls == "Dropout":
        return nn.Dropout(float(g("p", 0.5)))
    if cls == "Identity":
        return nn.Identity()
    if cls in ("View", "Reshape"):
        size = g("size")
        size = [int(v) for v in (size.tolist() if isinstance(size, np.ndarray) else _as_list(size))]
        return _View(size)
    raise NotImplementedError("Torch7 import: module %s is not supported" % (o.cls if isinstance(o, T7Object)
                                                                              else type(o)))


def load_torch7(path):
    """A ``.t7`` nn model -> torch.nn.Module (eval mode)."""
    return to_module(read_t7(path)).eval()


# ---------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------
class _Writer:
    def __init__(self):
        self.out = bytearray()
        self.idx = {}

    def int(self, v):
        self.out += struct.pack("<i", int(v))

    def long_(self, v):
        self.out += struct.pack("<q", int(v))

    def string(self, s):
        b = s.encode("latin-1") if isinstance(s, str) else s
        self.int(len(b))
        self.out += b

    def obj(self, v):
        if v is None:
            self.int(NIL)
        elif isinstance(v, bool):
            self.int(BOOLEAN)
            self.int(1 if v else 0)
        elif isinstance(v, (int, float)):
            self.int(NUMBER)
            self.out += struct.pack("<d", float(v))
        elif isinstance(v, str):
            self.int(STRING)
            self.string(v)
        elif isinstance(v, np.ndarray):
            self.int(TORCH)
            self.int(len(self.idx) + 1)
            self.idx[id(v)] = len(self.idx) + 1
            tcls = {np.dtype(np.float32): "torch.FloatTensor", np.dtype(np.float64): "torch.DoubleTensor",
                    np.dtype(np.int64): "torch.LongTensor"}[v.dtype]
            self.string("V 1")
            self.string(tcls)
            a = np.ascontiguousarray(v)
            self.int(a.ndim)
            for s in a.shape:
                self.long_(s)
            st = [int(x // a.itemsize) for x in a.strides] if a.ndim else []
            for s in st:
                self.long_(s)
            self.long_(1)
            self.int(TORCH)
            self.int(len(self.idx) + 1)
            self.idx[("s", id(v))] = len(self.idx) + 1
            self.string("V 1")
            self.string(tcls.replace("Tensor", "Storage"))
            self.long_(a.size)
            self.out += a.tobytes()
        elif isinstance(v, T7Object):
            self.int(TORCH)
            self.int(len(self.idx) + 1)
            self.idx[id(v)] = len(self.idx) + 1
            self.string("V 1")
            self.string(v.cls)
            self.obj(v.fields)
        elif isinstance(v, (dict, list)):
            d = v if isinstance(v, dict) else {float(i + 1): x for i, x in enumerate(v)}
            self.int(TABLE)
            self.int(len(self.idx) + 1)
            self.idx[id(v)] = len(self.idx) + 1
            self.int(len(d))
            for k, x in d.items():
                self.obj(k)
                self.obj(x)
        else:
            raise TypeError("write_t7: cannot serialise %r" % type(v))


def write_t7(obj, path):
    w = _Writer()
    w.obj(obj)
    with open(path, "wb") as f:
        f.write(bytes(w.out))


__all__ = ["read_t7", "load_torch7", "to_module", "write_t7", "T7Object"]
