"""TensorFlow GraphDef / SavedModel reader and a torch executor for it.

The reference runs TF graphs through libtensorflow over JNI (TFNet,
Zs/pipeline/api/net/TFNet.scala:57-620; TFNetForInference.scala for
SavedModels; Py/tfpark/tfnet.py:52-300). There is no TensorFlow in this
framework: the GraphDef protobuf is decoded with the safe wire-format codec
(zoo.utils.protobuf — nothing in the file is executed), and each TF op is
mapped onto a PyTorch-ROCm op, so a frozen graph runs on the MI355X (GEMMs
and convs land on hipBLASLt / MIOpen, everything else on torch's HIP
elementwise kernels) and is differentiable through torch autograd.

SavedModel variables are read from the TF tensor-bundle checkpoint
(``variables/variables.index`` is an SSTable of BundleEntryProto records,
``variables.data-*`` holds the raw little-endian tensor bytes).
"""
import json
import os
import struct

import numpy as np
import torch
import torch.nn.functional as F

from zoo.utils import protobuf as pb

# tensorflow/core/framework/types.proto
DTYPES = {
    1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 7: object,
    9: np.int64, 10: np.bool_, 14: "bfloat16", 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64,
}
_TORCH = {np.float32: torch.float32, np.float64: torch.float64, np.int32: torch.int32, np.uint8: torch.uint8,
          np.int16: torch.int16, np.int8: torch.int8, np.int64: torch.int64, np.bool_: torch.bool,
          np.float16: torch.float16, "bfloat16": torch.bfloat16}


def torch_dtype(dt):
    """TF DataType enum (ref-types have +100) -> torch dtype (None for strings)."""
    dt = int(dt) % 100
    npd = DTYPES.get(dt)
    if npd is None:
        raise NotImplementedError("TF dtype %d" % dt)
    if npd is object:
        return None
    if npd in (np.uint16, np.uint32, np.uint64):
        return torch.int64
    return _TORCH[npd]


# ---------------------------------------------------------------------------- protobuf decoding
def parse_shape(b):
    """TensorShapeProto -> list of dims (-1 unknown) or None for unknown rank."""
    g = pb.group(b)
    if g.get(3) and g[3][0][1]:
        return None
    dims = []
    for _w, d in g.get(2, []):
        dg = pb.group(d)
        dims.append(pb.as_int32(dg[1][0][1]) if 1 in dg else 0)
    return dims


def parse_tensor(b):
    """TensorProto -> numpy array (strings -> object array of bytes)."""
    g = pb.group(b)
    dt = g[1][0][1] if 1 in g else 1
    shape = parse_shape(g[2][0][1]) if 2 in g else []
    npd = DTYPES.get(dt)
    if npd is None:
        raise NotImplementedError("TF tensor dtype %d" % dt)
    n = int(np.prod(shape)) if shape else 1
    if npd is object:
        vals = [v for _w, v in g.get(8, [])]
        arr = np.empty(len(vals), dtype=object)
        arr[:] = vals
        if len(vals) == 1 and n > 1:
            arr = np.repeat(arr, n)
        return arr.reshape(shape)
    if 4 in g:  # tensor_content: raw little-endian bytes
        raw = g[4][0][1]
        if npd == "bfloat16":
            u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
            arr = u.view(np.float32)
        else:
            arr = np.frombuffer(raw, dtype=np.dtype(npd).newbyteorder("<")).astype(npd)
        return arr.reshape(shape).copy()
    if npd == np.float32:
        vals = pb.packed_floats(g.get(5, []))
    elif npd == np.float64:
        vals = pb.packed_doubles(g.get(6, []))
    elif npd in (np.int32, np.uint8, np.int16, np.int8, np.uint16):
        vals = np.asarray(pb.packed_varints(g.get(7, [])), dtype=np.int64)
    elif npd == np.int64:
        vals = np.asarray(pb.packed_varints(g.get(10, [])), dtype=np.int64)
    elif npd == np.bool_:
        vals = np.asarray(pb.packed_varints(g.get(11, [])), dtype=np.int64) != 0
    elif npd in (np.float16, "bfloat16"):
        h = np.asarray(pb.packed_varints(g.get(13, [])), dtype=np.uint16)
        vals = h.view(np.float16).astype(np.float32) if npd == np.float16 else \
            (h.astype(np.uint32) << 16).view(np.float32)
    elif npd in (np.uint32,):
        vals = np.asarray(pb.packed_varints(g.get(16, [])), dtype=np.int64)
    elif npd in (np.uint64,):
        vals = np.asarray(pb.packed_varints(g.get(17, [])), dtype=np.int64)
    else:
        vals = np.zeros(0)
    out_dt = np.float32 if npd == "bfloat16" else npd
    vals = np.asarray(vals).astype(out_dt)
    if vals.size == n:
        return vals.reshape(shape)
    if vals.size == 0:
        return np.zeros(shape, dtype=out_dt)
    # TF stores a repeated trailing value only once: broadcast the last element
    full = np.empty(n, dtype=out_dt)
    full[:vals.size] = vals
    full[vals.size:] = vals[-1]
    return full.reshape(shape)


def _parse_list(b):
    g = pb.group(b)
    if 2 in g:
        return [v for _w, v in g[2]]
    if 3 in g:
        return pb.packed_varints(g[3])
    if 4 in g:
        return [float(x) for x in pb.packed_floats(g[4])]
    if 5 in g:
        return [bool(x) for x in pb.packed_varints(g[5])]
    if 6 in g:
        return pb.packed_varints(g[6])
    if 7 in g:
        return [parse_shape(v) for _w, v in g[7]]
    if 8 in g:
        return [parse_tensor(v) for _w, v in g[8]]
    return []


def parse_attr(b):
    """AttrValue -> python value."""
    g = pb.group(b)
    if 1 in g:
        return _parse_list(g[1][0][1])
    if 2 in g:
        return g[2][0][1]
    if 3 in g:
        return pb.as_int32(g[3][0][1])
    if 4 in g:
        w, v = g[4][0]
        return pb.as_float32(w, v)
    if 5 in g:
        return bool(g[5][0][1])
    if 6 in g:
        return int(g[6][0][1])
    if 7 in g:
        return parse_shape(g[7][0][1])
    if 8 in g:
        return parse_tensor(g[8][0][1])
    if 9 in g:
        return pb.as_str(g[9][0][1])
    if 10 in g:   # func: NameAttrList (tf.data map / filter functions)
        return {"func": pb.as_str(pb.group(g[10][0][1])[1][0][1])}
    return None


class Node:
    __slots__ = ("name", "op", "inputs", "controls", "attr", "raw")

    def __init__(self, name, op, inputs, controls, attr, raw=None):
        self.name, self.op, self.inputs, self.controls, self.attr = name, op, inputs, controls, attr
        self.raw = raw   # the serialized NodeDef (kept for re-export, zoo.util.tf.export_tf)

    def s(self, key, default=""):
        v = self.attr.get(key, default)
        return pb.as_str(v) if isinstance(v, (bytes, bytearray)) else v

    def __repr__(self):
        return "Node(%s: %s <- %s)" % (self.name, self.op, self.inputs)


def parse_node(b):
    g = pb.group(b)
    name = pb.as_str(g[1][0][1])
    op = pb.as_str(g[2][0][1])
    inputs, controls = [], []
    for _w, v in g.get(3, []):
        s = pb.as_str(v)
        (controls if s.startswith("^") else inputs).append(s.lstrip("^"))
    attr = {}
    for _w, v in g.get(5, []):
        e = pb.group(v)
        attr[pb.as_str(e[1][0][1])] = parse_attr(e[2][0][1]) if 2 in e else None
    return Node(name, op, inputs, controls, attr, bytes(b))


def parse_graph_def(b):
    return [parse_node(v) for _w, v in pb.group(b).get(1, [])]


def split_name(t):
    """'scope/op:1' -> ('scope/op', 1); 'scope/op' -> ('scope/op', 0)."""
    if ":" in t:
        n, i = t.rsplit(":", 1)
        if i.isdigit():
            return n, int(i)
    return t, 0


# ---------------------------------------------------------------------------- SavedModel / bundle
def _sst_block_entries(data, off, size):
    blk = data[off:off + size]
    nrest = struct.unpack_from("<I", blk, size - 4)[0]
    end = size - 4 * (nrest + 1)
    i, key, out = 0, b"", []
    while i < end:
        shared, i = pb._varint(blk, i)
        nons, i = pb._varint(blk, i)
        vlen, i = pb._varint(blk, i)
        key = key[:shared] + blk[i:i + nons]
        i += nons
        out.append((bytes(key), bytes(blk[i:i + vlen])))
        i += vlen
    ctype = data[off + size]
    if ctype != 0:
        raise NotImplementedError("compressed SSTable block (type %d) in tensor bundle" % ctype)
    return out


def read_sstable(path):
    """LevelDB-format table (TF tensor-bundle index) -> [(key, value)]."""
    data = open(path, "rb").read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != 0xdb4775248b80fb57:
        raise ValueError("%s is not an SSTable" % path)
    foot = data[len(data) - 48:]
    i = 0
    _mo, i = pb._varint(foot, i)
    _ms, i = pb._varint(foot, i)
    io, i = pb._varint(foot, i)
    isz, i = pb._varint(foot, i)
    out = []
    for _k, handle in _sst_block_entries(data, io, isz):
        j = 0
        bo, j = pb._varint(handle, j)
        bs, j = pb._varint(handle, j)
        out.extend(_sst_block_entries(data, bo, bs))
    return out


def read_tensor_bundle(prefix, strict=True):
    """TF V2 checkpoint (``prefix.index`` + ``prefix.data-*``) -> {name: np.ndarray}.
    ``strict=False`` skips entries whose data shard is missing."""
    entries = read_sstable(prefix + ".index")
    shards = {}
    out = {}
    for key, val in entries:
        if not key:
            continue  # BundleHeaderProto
        g = pb.group(val)
        dt = g[1][0][1] if 1 in g else 1
        shape = parse_shape(g[2][0][1]) if 2 in g else []
        shard = g[3][0][1] if 3 in g else 0
        offset = g[4][0][1] if 4 in g else 0
        size = g[5][0][1] if 5 in g else 0
        if 7 in g:
            raise NotImplementedError("partitioned (sliced) variable %s" % key.decode())
        if shard not in shards:
            cands = [f for f in os.listdir(os.path.dirname(prefix) or ".")
                     if f.startswith(os.path.basename(prefix) + ".data-%05d-of-" % shard)]
            if not cands:
                if not strict:
                    shards[shard] = None
                    continue
                raise FileNotFoundError("bundle shard %d of %s" % (shard, prefix))
            shards[shard] = np.memmap(os.path.join(os.path.dirname(prefix), cands[0]), dtype=np.uint8, mode="r")
        if shards[shard] is None:
            continue
        raw = bytes(shards[shard][offset:offset + size])
        npd = DTYPES.get(dt)
        if npd is object:
            continue  # string variables are not used by inference graphs
        if npd == "bfloat16":
            arr = (np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16).view(np.float32)
        else:
            arr = np.frombuffer(raw, dtype=np.dtype(npd).newbyteorder("<")).astype(npd)
        out[key.decode()] = arr.reshape(shape).copy()
    return out


def load_saved_model(path, tag="serve"):
    """SavedModel dir -> (nodes, signature dict, variables dict)."""
    b = open(os.path.join(path, "saved_model.pb"), "rb").read()
    metas = [pb.group(v) for _w, v in pb.group(b).get(2, [])]
    chosen = None
    for m in metas:
        tags = [pb.as_str(v) for _w, v in pb.group(m[1][0][1]).get(4, [])] if 1 in m else []
        if tag is None or tag in tags:
            chosen = m
            break
    if chosen is None:
        raise ValueError("no MetaGraph with tag %r in %s" % (tag, path))
    nodes = parse_graph_def(chosen[2][0][1])
    sigs = {}
    for _w, v in chosen.get(5, []):
        e = pb.group(v)
        key = pb.as_str(e[1][0][1])
        sd = pb.group(e[2][0][1]) if 2 in e else {}

        def _tmap(entries):
            res = {}
            for _w2, vv in entries:
                me = pb.group(vv)
                ti = pb.group(me[2][0][1]) if 2 in me else {}
                res[pb.as_str(me[1][0][1])] = pb.as_str(ti[1][0][1]) if 1 in ti else None
            return res
        sigs[key] = {"inputs": _tmap(sd.get(1, [])), "outputs": _tmap(sd.get(2, [])),
                     "method": pb.as_str(sd[3][0][1]) if 3 in sd else ""}
    var_prefix = os.path.join(path, "variables", "variables")
    variables = read_tensor_bundle(var_prefix, strict=False) if os.path.exists(var_prefix + ".index") else {}
    return nodes, sigs, variables


# ---------------------------------------------------------------------------- executor
class _Dead:
    """Untaken branch of a Switch (TF dead tensor)."""


DEAD = _Dead()


def _same_pad(size, k, s, d=1):
    out = (size + s - 1) // s
    eff = (k - 1) * d + 1
    total = max((out - 1) * s + eff - size, 0)
    return total // 2, total - total // 2


def _nhwc(node):
    return node.s("data_format", "NHWC") in ("NHWC", "", None)


def _to_nchw(x, nhwc):
    return x.permute(0, 3, 1, 2) if nhwc else x


def _from_nchw(x, nhwc):
    return x.permute(0, 2, 3, 1).contiguous() if nhwc else x


def _hw(lst, nhwc):
    return (lst[1], lst[2]) if nhwc else (lst[2], lst[3])


def _conv2d_native(g, node, x, w):
    """NHWC Conv2D on the implicit-GEMM MFMA kernel (bf16 compute, fp32 out); the HWIO filter
    is packed once per weight version."""
    from zoo import ops
    kh, kw, cin, cout = w.shape
    strides = node.attr.get("strides", [1, 1, 1, 1])
    dil = node.attr.get("dilations", [1, 1, 1, 1])
    sh, sw, dh, dw = strides[1], strides[2], dil[1], dil[2]
    cin_p = cin if cin % 8 == 0 else (4 if cin <= 4 else ops.ceil8(cin))
    k_p = ops.ceil8(cout)
    key = (w.data_ptr(), w._version, tuple(w.shape))
    packed = g._packed.get(key)
    if packed is None:
        w4 = torch.zeros(k_p, kh, kw, cin_p, device=x.device)
        w4[:cout, :, :, :cin] = w.float().permute(3, 0, 1, 2)
        packed = g._packed[key] = ops.pack_weight(w4)
    xn = x
    pad = node.s("padding", "VALID")
    pt = pb_ = pl = pr = 0
    if pad == "SAME":
        pt, pb_ = _same_pad(x.shape[1], kh, sh, dh)
        pl, pr = _same_pad(x.shape[2], kw, sw, dw)
    elif pad == "EXPLICIT":
        ep = node.attr.get("explicit_paddings", [0] * 8)[2:6]
        pt, pb_, pl, pr = ep
    sym = pt == pb_ and pl == pr
    if not sym or cin_p != cin:
        xn = F.pad(xn, (0, cin_p - cin, 0 if sym else pl, 0 if sym else pr, 0 if sym else pt, 0 if sym else pb_))
    ph, pw = (pt, pl) if sym else (0, 0)
    g.native_calls += 1
    y = ops.conv2d_nhwc(xn.to(torch.bfloat16).contiguous(), packed, None, kernel=(kh, kw), stride=(sh, sw),
                        pad=[ph, pw], dil=(dh, dw), out_f32=True)
    return y[..., :cout]


def _conv2d(node, x, w, depthwise=False, g=None):
    nhwc = _nhwc(node)
    if (g is not None and g.native_bf16 and x.is_cuda and not depthwise and nhwc and w.dim() == 4
            and x.shape[-1] == w.shape[2]):
        return _conv2d_native(g, node, x, w)
    strides = node.attr.get("strides", [1, 1, 1, 1])
    dil = node.attr.get("dilations", [1, 1, 1, 1])
    sh, sw = _hw(strides, nhwc)
    dh, dw = _hw(dil, nhwc)
    xc = _to_nchw(x, nhwc)
    kh, kw = w.shape[0], w.shape[1]
    if depthwise:  # [kh, kw, in, mult] -> [in*mult, 1, kh, kw]
        cin, mult = w.shape[2], w.shape[3]
        wt = w.permute(2, 3, 0, 1).reshape(cin * mult, 1, kh, kw)
        groups = cin
    else:          # HWIO -> OIHW
        wt = w.permute(3, 2, 0, 1)
        groups = xc.shape[1] // w.shape[2]
    pad = node.s("padding", "VALID")
    if pad == "SAME":
        pt, pb_ = _same_pad(xc.shape[2], kh, sh, dh)
        pl, pr = _same_pad(xc.shape[3], kw, sw, dw)
        xc = F.pad(xc, (pl, pr, pt, pb_))
    elif pad == "EXPLICIT":
        ep = node.attr.get("explicit_paddings", [0] * 8)
        ep = ep[2:6] if nhwc else ep[4:8]
        xc = F.pad(xc, (ep[2], ep[3], ep[0], ep[1]))
    y = F.conv2d(xc, wt.to(xc.dtype), stride=(sh, sw), dilation=(dh, dw), groups=groups)
    return _from_nchw(y, nhwc)


def _pool(node, x, kind):
    nhwc = _nhwc(node)
    ks = node.attr.get("ksize", [1, 1, 1, 1])
    st = node.attr.get("strides", [1, 1, 1, 1])
    kh, kw = _hw(ks, nhwc)
    sh, sw = _hw(st, nhwc)
    xc = _to_nchw(x, nhwc)
    if node.s("padding", "VALID") == "SAME":
        pt, pb_ = _same_pad(xc.shape[2], kh, sh)
        pl, pr = _same_pad(xc.shape[3], kw, sw)
        if kind == "max":
            xc = F.pad(xc, (pl, pr, pt, pb_), value=float("-inf"))
            y = F.max_pool2d(xc, (kh, kw), (sh, sw))
        else:  # TF's SAME average excludes the padding from the divisor
            ones = torch.ones_like(xc[:1, :1])
            s = F.avg_pool2d(F.pad(xc, (pl, pr, pt, pb_)), (kh, kw), (sh, sw), divisor_override=1)
            c = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb_)), (kh, kw), (sh, sw), divisor_override=1)
            y = s / c
    else:
        y = F.max_pool2d(xc, (kh, kw), (sh, sw)) if kind == "max" else F.avg_pool2d(xc, (kh, kw), (sh, sw))
    return _from_nchw(y, nhwc)


def _axes(a, nd):
    a = a.reshape(-1).tolist() if torch.is_tensor(a) else ([a] if np.isscalar(a) else list(a))
    return [int(i) % nd if nd else 0 for i in a]


def _reduce(fn, node, x, axes):
    keep = bool(node.attr.get("keep_dims", node.attr.get("keepdims", False)))
    ax = _axes(axes, x.dim())
    if not ax:
        return x
    if fn == "mean":
        return x.float().mean(dim=ax, keepdim=keep).to(x.dtype) if not x.is_floating_point() else \
            x.mean(dim=ax, keepdim=keep)
    if fn == "sum":
        return x.sum(dim=ax, keepdim=keep)
    if fn == "prod":
        y = x
        for a in sorted(ax, reverse=True):
            y = y.prod(dim=a, keepdim=keep)
        return y
    if fn in ("max", "min", "all", "any"):
        y = x
        for a in sorted(ax, reverse=True):
            if fn == "max":
                y = y.amax(dim=a, keepdim=keep)
            elif fn == "min":
                y = y.amin(dim=a, keepdim=keep)
            elif fn == "all":
                y = y.all(dim=a, keepdim=keep)
            else:
                y = y.any(dim=a, keepdim=keep)
        return y
    raise NotImplementedError(fn)


def _ints(t):
    return [int(v) for v in (t.reshape(-1).tolist() if torch.is_tensor(t) else np.asarray(t).reshape(-1))]


def _strided_slice(node, x, begin, end, strides):
    begin, end, strides = _ints(begin), _ints(end), _ints(strides)
    bm = int(node.attr.get("begin_mask", 0))
    em = int(node.attr.get("end_mask", 0))
    elm = int(node.attr.get("ellipsis_mask", 0))
    nam = int(node.attr.get("new_axis_mask", 0))
    sam = int(node.attr.get("shrink_axis_mask", 0))
    idx = []
    n_spec = len(begin)
    # number of real dims covered by explicit (non-ellipsis, non-new-axis) specs
    explicit = sum(1 for i in range(n_spec) if not (elm >> i) & 1 and not (nam >> i) & 1)
    dim = 0
    for i in range(n_spec):
        if (elm >> i) & 1:
            fill = x.dim() - explicit - dim
            idx.extend([slice(None)] * fill)
            dim += fill
            continue
        if (nam >> i) & 1:
            idx.append(None)
            continue
        size = x.shape[dim]
        if (sam >> i) & 1:
            b = begin[i]
            idx.append(b + size if b < 0 else b)
        else:
            s = strides[i]
            b = None if (bm >> i) & 1 else begin[i]
            e = None if (em >> i) & 1 else end[i]
            if s < 0:
                # python slicing with negative step over a flipped view
                b = size - 1 if b is None else (b + size if b < 0 else b)
                e = -1 if e is None else (e + size if e < 0 else e)
                ln = max(0, (b - e + (-s) - 1) // (-s))
                idx.append(("rev", b, ln, -s))
                dim += 1
                continue
            idx.append(slice(b, e, s))
        dim += 1
    out = x
    # apply: basic indexing for everything but reversed slices
    basic, revs = [], []
    for k, it in enumerate(idx):
        if isinstance(it, tuple):
            basic.append(slice(None))
            revs.append((k, it))
        else:
            basic.append(it)
    out = out[tuple(basic)] if basic else out
    for k, (_tag, b, ln, st) in revs:
        # position of dim k in `out` after shrink/new-axis handling
        pos = sum(1 for it in idx[:k] if not isinstance(it, int) or isinstance(it, bool))
        ind = torch.arange(b, b - ln * st, -st, device=out.device)
        out = out.index_select(pos, ind)
    return out


def _np_bytes_to_str(v):
    return v.decode("utf-8") if isinstance(v, (bytes, bytearray)) else str(v)


class TFGraph:
    """Executes a set of TF nodes with torch. ``params`` maps variable / const
    names to tensors (nn.Parameters or buffers owned by the caller)."""

    def __init__(self, nodes, values):
        self.nodes = {n.name: n for n in nodes}
        self.values = values  # name -> torch tensor (Const / variables)
        # native bf16 execution of Conv2D / MatMul on the GPU (MFMA kernels; opt-in because the
        # graph's own dtype is fp32): TFNet.use_native_kernels(True) or ZOO_TF_NATIVE_BF16=1
        self.native_bf16 = os.environ.get("ZOO_TF_NATIVE_BF16", "0") == "1"
        self._packed = {}
        self.native_calls = 0

    def needed(self, fetches, feeds=()):
        feed_nodes = {split_name(f)[0] for f in feeds}
        seen, order = set(), []

        def visit(name):
            stack = [(name, False)]
            while stack:
                n, done = stack.pop()
                if done:
                    order.append(n)
                    continue
                if n in seen:
                    continue
                seen.add(n)
                stack.append((n, True))
                if n in feed_nodes:
                    continue
                node = self.nodes.get(n)
                if node is None:
                    raise KeyError("tensor %s not in graph" % n)
                for i in node.inputs:
                    stack.append((split_name(i)[0], False))
        for f in fetches:
            visit(split_name(f)[0])
        return order

    def run(self, feeds, fetches):
        order = self.needed(fetches, feeds)
        env = {}
        feed_by_node = {}
        for k, v in feeds.items():
            n, i = split_name(k)
            feed_by_node.setdefault(n, {})[i] = v
        for name in order:
            if name in feed_by_node:
                fv = feed_by_node[name]
                env[name] = [fv.get(i) for i in range(max(fv) + 1)]
                continue
            node = self.nodes[name]
            ins = []
            for t in node.inputs:
                n, i = split_name(t)
                outs = env[n]
                ins.append(outs[i] if i < len(outs) else None)
            env[name] = self._exec(node, ins)
        res = []
        for f in fetches:
            n, i = split_name(f)
            v = env[n][i]
            if v is DEAD:
                raise RuntimeError("fetched tensor %s is on an untaken branch" % f)
            res.append(v)
        return res

    # ------------------------------------------------------------------
    def _exec(self, node, ins):
        op = node.op
        if op != "Merge" and any(v is DEAD for v in ins):
            return [DEAD] * 2
        fn = _OPS.get(op)
        if fn is None:
            raise NotImplementedError("TF op %s (node %s) is not supported" % (op, node.name))
        out = fn(self, node, *ins)
        return out if isinstance(out, list) else [out]


def _t(v, like=None):
    if torch.is_tensor(v):
        return v
    dev = like.device if torch.is_tensor(like) else None
    return torch.as_tensor(np.asarray(v), device=dev)


def _bin(f):
    def run(g, node, a, b):
        a, b = _t(a), _t(b)
        if a.device != b.device:
            b = b.to(a.device) if b.dim() == 0 or a.numel() >= b.numel() else b
            a = a.to(b.device)
        return f(a, b)
    return run


def _const(g, node):
    return g.values[node.name]


def _var(g, node):
    key = node.s("shared_name") or node.name
    if key in g.values:
        return g.values[key]
    return g.values[node.name]


def _placeholder_default(g, node, x):
    return x


def _switch(g, node, x, pred):
    p = bool(_t(pred).reshape(-1)[0].item())
    return [DEAD, x] if p else [x, DEAD]


def _merge(g, node, *ins):
    for i, v in enumerate(ins):
        if v is not DEAD and v is not None:
            return [v, torch.tensor(i, dtype=torch.int32)]
    return [DEAD, DEAD]


def _matmul(g, node, a, b):
    if node.attr.get("transpose_a", False):
        a = a.transpose(-1, -2)
    if node.attr.get("transpose_b", False):
        b = b.transpose(-1, -2)
    if g is not None and g.native_bf16 and a.is_cuda and a.dim() == 2 and b.dim() == 2 and a.is_floating_point():
        from zoo import ops
        g.native_calls += 1
        return ops.linear(a.float(), b.t().float().contiguous()).float()
    return torch.matmul(a, b.to(a.dtype))


def _batch_matmul(g, node, a, b):
    if node.attr.get("adj_x", False):
        a = a.transpose(-1, -2)
    if node.attr.get("adj_y", False):
        b = b.transpose(-1, -2)
    return torch.matmul(a, b.to(a.dtype))


def _bias_add(g, node, x, b):
    if node.s("data_format", "NHWC") == "NCHW" and x.dim() >= 3:
        return x + b.to(x.dtype).reshape([1, -1] + [1] * (x.dim() - 2))
    return x + b.to(x.dtype)


def _bias_add_grad(g, node, dy):
    if node.s("data_format", "NHWC") == "NCHW" and dy.dim() >= 3:
        return dy.sum(dim=[0] + list(range(2, dy.dim())))
    return dy.reshape(-1, dy.shape[-1]).sum(0)


def _fused_bn(g, node, x, scale, offset, mean, var):
    eps = float(node.attr.get("epsilon", 1e-3))
    nhwc = _nhwc(node)
    shp = [1, 1, 1, -1] if nhwc else [1, -1, 1, 1]
    if node.attr.get("is_training", True):
        dims = [0, 1, 2] if nhwc else [0, 2, 3]
        m = x.mean(dim=dims)
        v = x.var(dim=dims, unbiased=False)
    else:
        m, v = mean, var
    y = (x - m.reshape(shp)) * torch.rsqrt(v.reshape(shp) + eps) * scale.reshape(shp) + offset.reshape(shp)
    return [y, m, v, m, v, v]


def _reshape(g, node, x, shape):
    return x.reshape(_ints(shape))


def _concat(g, node, *ins):
    if node.op == "Concat":
        axis, vals = ins[0], ins[1:]
    else:
        axis, vals = ins[-1], ins[:-1]
    vals = [_t(v) for v in vals]
    ax = int(_t(axis).item()) % vals[0].dim()
    return torch.cat([v.to(vals[0].dtype) for v in vals], dim=ax)


def _pack(g, node, *ins):
    vals = [_t(v) for v in ins]
    ax = int(node.attr.get("axis", 0))
    ax = ax % (vals[0].dim() + 1)
    return torch.stack([v.to(vals[0].dtype) for v in vals], dim=ax)


def _unpack(g, node, x):
    ax = int(node.attr.get("axis", 0)) % x.dim()
    return list(torch.unbind(x, dim=ax))


def _shape(g, node, x):
    dt = torch_dtype(node.attr.get("out_type", 3)) or torch.int32
    return torch.tensor(list(x.shape), dtype=dt)


def _cast(g, node, x):
    dt = torch_dtype(node.attr.get("DstT", 1))
    if dt is None:
        raise NotImplementedError("Cast to string")
    return _t(x).to(dt)


def _fill(g, node, dims, value):
    v = _t(value)
    return torch.full(_ints(dims), v.item(), dtype=v.dtype, device=v.device)


def _range(g, node, start, limit, delta):
    s, l_, d = _t(start), _t(limit), _t(delta)
    return torch.arange(s.item(), l_.item(), d.item(), dtype=s.dtype)


def _squeeze(g, node, x):
    dims = node.attr.get("squeeze_dims", []) or []
    if not dims:
        return x.squeeze()
    for d in sorted([d % x.dim() for d in dims], reverse=True):
        x = x.squeeze(d)
    return x


def _expand_dims(g, node, x, dim):
    d = int(_t(dim).reshape(-1)[0].item())
    x = _t(x)
    return x.unsqueeze(d if d >= 0 else d + x.dim() + 1)


def _transpose(g, node, x, perm):
    return x.permute(*_ints(perm))


def _gather(g, node, params, indices, axis=None):
    ax = 0 if axis is None else int(_t(axis).item())
    idx = _t(indices).long()
    ax %= params.dim()
    out = params.index_select(ax, idx.reshape(-1).to(params.device))
    shp = list(params.shape[:ax]) + list(idx.shape) + list(params.shape[ax + 1:])
    return out.reshape(shp)


def _slice(g, node, x, begin, size):
    b, s = _ints(begin), _ints(size)
    idx = tuple(slice(bb, None if ss == -1 else bb + ss) for bb, ss in zip(b, s))
    return x[idx]


def _split(g, node, axis, x):
    n = int(node.attr.get("num_split", 1))
    ax = int(_t(axis).item()) % x.dim()
    return list(torch.chunk(x, n, dim=ax))


def _splitv(g, node, x, sizes, axis):
    ax = int(_t(axis).item()) % x.dim()
    sz = _ints(sizes)
    if -1 in sz:
        k = sz.index(-1)
        sz[k] = x.shape[ax] - (sum(sz) + 1)
    return list(torch.split(x, sz, dim=ax))


def _pad(g, node, x, paddings, value=None):
    p = _t(paddings).reshape(-1, 2).tolist()
    flat = []
    for lo, hi in reversed(p):
        flat += [int(lo), int(hi)]
    v = 0.0 if value is None else float(_t(value).item())
    return F.pad(x, flat, value=v)


def _tile(g, node, x, mult):
    return x.repeat(*_ints(mult))


def _argmax(g, node, x, axis):
    dt = torch_dtype(node.attr.get("output_type", 9)) or torch.int64
    return x.argmax(dim=int(_t(axis).item())).to(dt)


def _argmin(g, node, x, axis):
    dt = torch_dtype(node.attr.get("output_type", 9)) or torch.int64
    return x.argmin(dim=int(_t(axis).item())).to(dt)


def _select(g, node, c, a, b):
    c = _t(c).bool()
    if node.op == "Select" and c.dim() == 1 and a.dim() > 1:
        c = c.reshape([-1] + [1] * (a.dim() - 1))
    return torch.where(c, a, b)


def _softmax(g, node, x):
    return torch.softmax(x, dim=-1)


def _log_softmax(g, node, x):
    return torch.log_softmax(x, dim=-1)


def _leaky(g, node, x):
    return F.leaky_relu(x, float(node.attr.get("alpha", 0.2)))


def _div_no_nan(a, b):
    return torch.where(b == 0, torch.zeros_like(a / torch.where(b == 0, torch.ones_like(b), b)),
                       a / torch.where(b == 0, torch.ones_like(b), b))


def _string_to_number(g, node, x):
    dt = torch_dtype(node.attr.get("out_type", 1))
    arr = np.asarray(x, dtype=object)
    vals = np.vectorize(lambda s: float(_np_bytes_to_str(s)), otypes=[np.float64])(arr) if arr.size else arr
    return torch.as_tensor(np.asarray(vals, dtype=np.float64)).to(dt)


def _random_uniform(g, node, shape):
    dt = torch_dtype(node.attr.get("dtype", 1))
    return torch.rand(_ints(shape), dtype=dt)


def _random_normal(g, node, shape):
    dt = torch_dtype(node.attr.get("dtype", 1))
    z = torch.randn(_ints(shape), dtype=dt)
    if node.op == "TruncatedNormal":
        z = torch.fmod(z, 2.0)
    return z


def _noop(g, node, *ins):
    return [None]


def _identity_n(g, node, *ins):
    return list(ins)


def _lrn(g, node, x):
    r = int(node.attr.get("depth_radius", 5))
    bias = float(node.attr.get("bias", 1.0))
    alpha = float(node.attr.get("alpha", 1.0))
    beta = float(node.attr.get("beta", 0.5))
    sq = (x * x).permute(0, 3, 1, 2).unsqueeze(1)
    s = F.avg_pool3d(F.pad(sq, (0, 0, 0, 0, r, r)), (2 * r + 1, 1, 1), stride=1, divisor_override=1)
    s = s.squeeze(1).permute(0, 2, 3, 1)
    return x / (bias + alpha * s) ** beta


_OPS = {
    "Const": _const, "VariableV2": _var, "Variable": _var, "VarHandleOp": _var,
    "Placeholder": lambda g, n: (_ for _ in ()).throw(ValueError("placeholder %s was not fed" % n.name)),
    "PlaceholderWithDefault": _placeholder_default,
    "Identity": lambda g, n, x, *c: x, "StopGradient": lambda g, n, x: x.detach() if torch.is_tensor(x) else x,
    "PreventGradient": lambda g, n, x: x, "Snapshot": lambda g, n, x: x, "ReadVariableOp": lambda g, n, x: x,
    "IdentityN": _identity_n, "NoOp": _noop, "Assert": _noop, "Switch": _switch, "Merge": _merge,
    "Add": _bin(torch.add), "AddV2": _bin(torch.add), "Sub": _bin(torch.sub), "Mul": _bin(torch.mul),
    "RealDiv": _bin(torch.div), "Div": _bin(lambda a, b: torch.div(a, b) if a.is_floating_point()
                                              else torch.div(a, b, rounding_mode="trunc")),
    "FloorDiv": _bin(lambda a, b: torch.div(a, b, rounding_mode="floor")), "FloorMod": _bin(torch.remainder),
    "Maximum": _bin(torch.maximum), "Minimum": _bin(torch.minimum), "Pow": _bin(torch.pow),
    "SquaredDifference": _bin(lambda a, b: (a - b) * (a - b)), "DivNoNan": _bin(_div_no_nan),
    "Equal": _bin(torch.eq), "NotEqual": _bin(torch.ne), "Less": _bin(torch.lt), "LessEqual": _bin(torch.le),
    "Greater": _bin(torch.gt), "GreaterEqual": _bin(torch.ge), "LogicalAnd": _bin(torch.logical_and),
    "LogicalOr": _bin(torch.logical_or), "LogicalNot": lambda g, n, x: torch.logical_not(x),
    "AddN": lambda g, n, *xs: sum(xs[1:], xs[0]),
    "Neg": lambda g, n, x: -x, "Abs": lambda g, n, x: x.abs(), "Exp": lambda g, n, x: x.exp(),
    "Log": lambda g, n, x: x.log(), "Log1p": lambda g, n, x: x.log1p(), "Sqrt": lambda g, n, x: x.sqrt(),
    "Rsqrt": lambda g, n, x: x.rsqrt(), "Square": lambda g, n, x: x * x, "Reciprocal": lambda g, n, x: 1.0 / x,
    "Inv": lambda g, n, x: 1.0 / x, "Floor": lambda g, n, x: x.floor(), "Ceil": lambda g, n, x: x.ceil(),
    "Round": lambda g, n, x: x.round(), "Sign": lambda g, n, x: x.sign(), "Tanh": lambda g, n, x: x.tanh(),
    "Sigmoid": lambda g, n, x: x.sigmoid(), "Relu": lambda g, n, x: F.relu(x), "Relu6": lambda g, n, x: F.relu6(x),
    "Elu": lambda g, n, x: F.elu(x), "Selu": lambda g, n, x: F.selu(x), "Softplus": lambda g, n, x: F.softplus(x),
    "Softsign": lambda g, n, x: F.softsign(x), "LeakyRelu": _leaky, "Erf": lambda g, n, x: torch.erf(x),
    "Sin": lambda g, n, x: x.sin(), "Cos": lambda g, n, x: x.cos(),
    "ReluGrad": lambda g, n, dy, x: dy * (x > 0).to(dy.dtype),
    "Relu6Grad": lambda g, n, dy, x: dy * ((x > 0) & (x < 6)).to(dy.dtype),
    "SigmoidGrad": lambda g, n, y, dy: dy * y * (1 - y), "TanhGrad": lambda g, n, y, dy: dy * (1 - y * y),
    "BiasAddGrad": _bias_add_grad,
    "MatMul": _matmul, "BatchMatMul": _batch_matmul, "BatchMatMulV2": _batch_matmul,
    "BiasAdd": _bias_add, "BiasAddV1": _bias_add,
    "Conv2D": lambda g, n, x, w: _conv2d(n, x, w, g=g),
    "DepthwiseConv2dNative": lambda g, n, x, w: _conv2d(n, x, w, depthwise=True),
    "MaxPool": lambda g, n, x: _pool(n, x, "max"), "AvgPool": lambda g, n, x: _pool(n, x, "avg"),
    "FusedBatchNorm": _fused_bn, "FusedBatchNormV2": _fused_bn, "FusedBatchNormV3": _fused_bn, "LRN": _lrn,
    "Softmax": _softmax, "LogSoftmax": _log_softmax,
    "Shape": _shape, "Size": lambda g, n, x: torch.tensor(x.numel(), dtype=torch.int32),
    "Rank": lambda g, n, x: torch.tensor(x.dim(), dtype=torch.int32),
    "Reshape": _reshape, "Squeeze": _squeeze, "ExpandDims": _expand_dims, "ConcatV2": _concat, "Concat": _concat,
    "Pack": _pack, "Unpack": _unpack, "StridedSlice": lambda g, n, x, b, e, s: _strided_slice(n, x, b, e, s),
    "Slice": _slice, "Transpose": _transpose, "Fill": _fill, "Range": _range, "Tile": _tile,
    "ZerosLike": lambda g, n, x: torch.zeros_like(x), "OnesLike": lambda g, n, x: torch.ones_like(x),
    "GatherV2": _gather, "Gather": _gather, "ResourceGather": _gather, "Split": _split, "SplitV": _splitv,
    "Pad": _pad, "PadV2": _pad, "Cast": _cast, "ArgMax": _argmax, "ArgMin": _argmin,
    "Select": _select, "SelectV2": _select,
    "Mean": lambda g, n, x, a: _reduce("mean", n, x, a), "Sum": lambda g, n, x, a: _reduce("sum", n, x, a),
    "Max": lambda g, n, x, a: _reduce("max", n, x, a), "Min": lambda g, n, x, a: _reduce("min", n, x, a),
    "Prod": lambda g, n, x, a: _reduce("prod", n, x, a), "All": lambda g, n, x, a: _reduce("all", n, x, a),
    "Any": lambda g, n, x, a: _reduce("any", n, x, a),
    "StringToNumber": _string_to_number, "RandomUniform": _random_uniform,
    "RandomStandardNormal": _random_normal, "TruncatedNormal": _random_normal,
}


def supported_ops():
    return sorted(k for k in _OPS)


def graph_meta(folder):
    with open(os.path.join(folder, "graph_meta.json")) as f:
        return json.load(f)


__all__ = ["TFGraph", "parse_graph_def", "load_saved_model", "read_tensor_bundle", "read_sstable",
           "parse_tensor", "split_name", "torch_dtype", "supported_ops", "graph_meta"]
