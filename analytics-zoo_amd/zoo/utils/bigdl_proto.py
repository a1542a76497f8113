"""BigDL ``.model`` protobuf codec (the format of Net.loadBigDL / saveModule).

Schema (BigDL serialization ``bigdl.proto``, observed on the reference
fixture zoo/src/test/resources/models/bigdl/bigdl_lenet.model):

  BigDLModule: 1 name, 2 subModules*, 3 weight, 4 bias, 5 preModules*,
               6 nextModules*, 7 moduleType, 8 attr (map<string, AttrValue>),
               9 version, 10 train, 11 namePostfix, 12 id, 16 parameters*
  BigDLTensor: 1 datatype, 2 size*, 3 stride*, 4 offset (1-based),
               5 dimension, 6 nElements, 7 isScalar, 8 storage, 9 id
  TensorStorage: 1 datatype, 2 float_data*, 3 double_data*, 4 bool_data*,
               5 string_data*, 6 int_data*, 7 long_data*, 8 bytes_data*, 9 id
  AttrValue:   1 dataType, 2 subType, then one of 3 int32, 4 int64, 5 float,
               6 double, 7 string, 8 bool, 9 regularizer, 10 tensor,
               11 variableFormat, 12 initMethod, 13 module, 14 nameAttrList,
               15 arrayValue, 16 dataFormat, 17 custom, 18 shape
  ArrayValue:  1 size, 2 datatype, 3 i32*, 4 i64*, 5 flt*, 6 dbl*, 7 str*,
               8 boolean*, 10 tensor*, 14 module*
  NameAttrList: 1 name, 2 attr (map<string, AttrValue>)

Tensor data lives once in the top module's ``global_storage`` attr
(NameAttrList keyed by tensor id); module tensors reference it by storage id.
Decoding builds plain Python objects only.
"""
import numpy as np

from zoo.utils.protobuf import (as_float32, as_int32, as_str, enc_bytes, enc_float, enc_int, enc_packed_floats,
                                enc_packed_doubles,
                                enc_packed_ints, fields, group, packed_doubles, packed_floats, packed_varints,
                                pb_fields_py)  # noqa: F401  (pb_fields_py re-exported for tensorboard)

INT32, INT64, FLOAT, DOUBLE, STRING, BOOL, CHAR, SHORT, BYTES, REGULARIZER, TENSOR, VARIABLE_FORMAT, \
    INITMETHOD, MODULE, NAME_ATTR_LIST, ARRAY_VALUE, DATA_FORMAT, CUSTOM, SHAPE = range(19)


class TensorRef:
    """A module tensor: geometry + the storage/tensor ids it points at."""

    def __init__(self, size, stride, offset, n, storage_id, tensor_id, data=None):
        self.size, self.stride, self.offset, self.n = size, stride, offset, n
        self.storage_id, self.tensor_id, self.data = storage_id, tensor_id, data

    def materialize(self, storages, native=False):
        """numpy array of the tensor: float32 by default; ``native`` keeps the storage dtype
        (int32 / int64 / float64 storages round-trip exactly)."""
        data = self.data
        if data is None:
            data = storages.get(self.storage_id)
        if data is None:
            data = storages.get(("tensor", self.tensor_id))
        if data is None:
            raise ValueError("BigDL tensor %s: storage %s not found" % (self.tensor_id, self.storage_id))
        out_dt = data.dtype if native else np.float32
        if not self.size:
            return np.asarray(data[self.offset - 1:self.offset], dtype=out_dt).reshape(())
        off = max(self.offset - 1, 0)
        strides = self.stride or list(np.cumprod(([1] + self.size[::-1])[:-1])[::-1])
        itemsize = data.dtype.itemsize
        view = np.lib.stride_tricks.as_strided(data[off:], shape=tuple(self.size),
                                               strides=tuple(int(s) * itemsize for s in strides))
        return np.array(view, dtype=out_dt)


def _storage(b):
    g = group(b)
    sid = as_int32(g[9][0][1]) if 9 in g else None
    if 2 in g:
        data = packed_floats(g[2])
    elif 3 in g:
        data = packed_doubles(g[3])
    elif 6 in g:
        data = np.asarray(packed_varints(g[6]), dtype=np.int32)
    elif 7 in g:
        data = np.asarray(packed_varints(g[7]), dtype=np.int64)
    else:
        data = None
    return sid, data


def decode_tensor(b):
    g = group(b)
    size = packed_varints(g.get(2, []))
    stride = packed_varints(g.get(3, []))
    offset = as_int32(g[4][0][1]) if 4 in g else 1
    n = as_int32(g[6][0][1]) if 6 in g else int(np.prod(size)) if size else 1
    tid = as_int32(g[9][0][1]) if 9 in g else None
    sid, data = _storage(g[8][0][1]) if 8 in g else (None, None)
    return TensorRef(size, stride, offset, n, sid, tid, data)


def decode_attr(b):
    g = group(b)
    dt = g[1][0][1] if 1 in g else None
    for f in range(3, 19):
        if f not in g:
            continue
        w, v = g[f][0]
        if f == 3:
            return as_int32(v)
        if f == 4:
            return as_int32(v)
        if f == 5:
            return as_float32(w, v)
        if f == 6:
            return as_float32(w, v)
        if f == 7:
            return as_str(v)
        if f == 8:
            return bool(v)
        if f == 10:
            return decode_tensor(v)
        if f == 13:
            return decode_module(v)
        if f == 14:
            return decode_name_attr_list(v)
        if f == 15:
            return decode_array(v)
        if f == 16:
            return {0: "NCHW", 1: "NHWC"}.get(v, v) if w == 0 else v
        if f == 18:
            return decode_shape(v)
        return ("opaque", f, v)
    # proto3 default values are omitted: decode by the declared type
    return {INT32: 0, INT64: 0, FLOAT: 0.0, DOUBLE: 0.0, STRING: "", BOOL: False, DATA_FORMAT: "NCHW"}.get(dt)


def decode_shape(b):
    g = group(b)
    return {"type": g[1][0][1] if 1 in g else 0, "ssize": as_int32(g[2][0][1]) if 2 in g else 0,
            "shape": packed_varints(g.get(3, [])), "shapes": [decode_shape(v) for _, v in g.get(4, [])]}


def decode_array(b):
    g = group(b)
    for f, conv in ((3, None), (4, None), (5, "f"), (6, "d"), (7, "s"), (8, "b"), (10, "t"), (14, "m")):
        if f not in g:
            continue
        if conv is None:
            return packed_varints(g[f])
        if conv == "f":
            return packed_floats(g[f]).tolist()
        if conv == "d":
            return packed_doubles(g[f]).tolist()
        if conv == "s":
            return [as_str(v) for _, v in g[f]]
        if conv == "b":
            return [bool(x) for x in packed_varints(g[f])]
        if conv == "t":
            return [decode_tensor(v) for _, v in g[f]]
        if conv == "m":
            return [decode_module(v) for _, v in g[f]]
    return []


def decode_name_attr_list(b):
    g = group(b)
    name = as_str(g[1][0][1]) if 1 in g else ""
    attrs = {}
    for _, entry in g.get(2, []):
        kv = group(entry)
        key = as_str(kv[1][0][1]) if 1 in kv else ""
        attrs[key] = decode_attr(kv[2][0][1]) if 2 in kv else None
    return {"name": name, "attr": attrs}


class BigDLModuleSpec:
    def __init__(self):
        self.name = ""
        self.type = ""
        self.submodules = []
        self.weight = None
        self.bias = None
        self.parameters = []
        self.pre = []
        self.next = []
        self.attr = {}
        self.train = False
        self.version = ""
        self.name_postfix = ""

    @property
    def effective_name(self):
        """BigDL's default module name: class name + namePostfix when ``name`` is empty."""
        return self.name or (self.short_type + self.name_postfix)

    @property
    def short_type(self):
        return self.type.split(".")[-1]

    def __repr__(self):
        return "BigDLModuleSpec(%s:%s, %d subs)" % (self.name, self.short_type, len(self.submodules))


def decode_module(b):
    m = BigDLModuleSpec()
    for f, w, v in fields(b):
        if f == 1:
            m.name = as_str(v)
        elif f == 2:
            m.submodules.append(decode_module(v))
        elif f == 3:
            m.weight = decode_tensor(v)
        elif f == 4:
            m.bias = decode_tensor(v)
        elif f == 5:
            m.pre.append(as_str(v))
        elif f == 6:
            m.next.append(as_str(v))
        elif f == 7:
            m.type = as_str(v)
        elif f == 8:
            kv = group(v)
            key = as_str(kv[1][0][1]) if 1 in kv else ""
            m.attr[key] = decode_attr(kv[2][0][1]) if 2 in kv else None
        elif f == 9:
            m.version = as_str(v)
        elif f == 10:
            m.train = bool(v)
        elif f == 11:
            m.name_postfix = as_str(v)
        elif f == 16:
            m.parameters.append(decode_tensor(v))
    return m


def collect_storages(root):
    """storage id -> flat data, from the ``global_storage`` attr and inline storages."""
    out = {}
    gs = root.attr.get("global_storage")
    if isinstance(gs, dict):
        for key, t in gs["attr"].items():
            if isinstance(t, TensorRef) and t.data is not None:
                if t.storage_id is not None:
                    out[t.storage_id] = t.data
                out[("tensor", t.tensor_id)] = t.data

    def visit(m):
        for t in [m.weight, m.bias] + list(m.parameters):
            if isinstance(t, TensorRef) and t.data is not None and t.storage_id is not None:
                out.setdefault(t.storage_id, t.data)
        for s in m.submodules:
            visit(s)
    visit(root)
    return out


def load_bigdl_spec(path):
    with open(path, "rb") as f:
        data = f.read()
    root = decode_module(data)
    return root, collect_storages(root)


# ---- encoder (saveModule in the same format) ------------------------------------------
_ids = iter(range(1000, 1 << 30))


def _enc_attr_value(v):
    if isinstance(v, bool):
        return enc_int(1, BOOL) + enc_int(8, int(v))
    if isinstance(v, int):
        return enc_int(1, INT32) + enc_int(3, v)
    if isinstance(v, float):
        return enc_int(1, FLOAT) + enc_float(5, v)
    if isinstance(v, str):
        return enc_int(1, STRING) + enc_bytes(7, v)
    if isinstance(v, (list, tuple)) and all(isinstance(x, int) for x in v):
        arr = enc_int(1, len(v)) + enc_int(2, INT32) + enc_packed_ints(3, v)
        return enc_int(1, ARRAY_VALUE) + enc_bytes(15, arr)
    if isinstance(v, dict) and "edges" in v:
        body = enc_bytes(1, v["name"])
        for pre in v["edges"]:
            entry = enc_bytes(1, pre) + enc_bytes(2, enc_int(1, INT32) + enc_int(3, -1))
            body += enc_bytes(2, entry)
        return enc_int(1, NAME_ATTR_LIST) + enc_bytes(14, body)
    raise TypeError("cannot encode attr %r" % (v,))


def _enc_tensor(arr, storages):
    arr = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
    tid, sid = next(_ids), next(_ids)
    storages.append((tid, sid, arr))
    st = enc_int(1, FLOAT) + enc_int(9, sid)
    body = enc_int(1, FLOAT) + enc_packed_ints(2, arr.shape)
    strides = [s // 4 for s in arr.strides]
    body += enc_packed_ints(3, strides) + enc_int(4, 1) + enc_int(5, arr.ndim) + enc_int(6, arr.size)
    body += enc_bytes(8, st) + enc_int(9, tid)
    return body


def encode_module(spec, storages=None, top=True):
    """spec: dict(name, type, attr{}, weight, bias, submodules[], pre[], next[])."""
    storages = [] if storages is None else storages
    out = enc_bytes(1, spec["name"])
    for s in spec.get("submodules", []):
        out += enc_bytes(2, encode_module(s, storages, False))
    if spec.get("weight") is not None:
        out += enc_bytes(3, _enc_tensor(spec["weight"], storages))
    if spec.get("bias") is not None:
        out += enc_bytes(4, _enc_tensor(spec["bias"], storages))
    for p in spec.get("pre", []):
        out += enc_bytes(5, p)
    for p in spec.get("next", []):
        out += enc_bytes(6, p)
    out += enc_bytes(7, spec["type"])
    for k, v in spec.get("attr", {}).items():
        out += enc_bytes(8, enc_bytes(1, k) + enc_bytes(2, _enc_attr_value(v)))
    out += enc_bytes(9, "0.10.0") + enc_int(10, 1)
    if top:
        body = enc_bytes(1, "global_storage")
        for tid, sid, arr in storages:
            st = enc_int(1, FLOAT) + enc_packed_floats(2, arr.reshape(-1)) + enc_int(9, sid)
            t = enc_int(1, FLOAT) + enc_packed_ints(2, arr.shape) + enc_int(4, 1) + enc_int(6, arr.size) + \
                enc_bytes(8, st) + enc_int(9, tid)
            av = enc_int(1, TENSOR) + enc_bytes(10, t)
            body += enc_bytes(2, enc_bytes(1, str(tid)) + enc_bytes(2, av))
        out += enc_bytes(8, enc_bytes(1, "global_storage") + enc_bytes(2, enc_int(1, NAME_ATTR_LIST) +
                                                                      enc_bytes(14, body)))
    return out
