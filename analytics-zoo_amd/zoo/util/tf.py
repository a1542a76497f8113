"""Py/util/tf.py: ``export_tf`` freezes a graph into the folder layout TFNet loads
(``frozen_inference_graph.pb`` + ``graph_meta.json``).

The reference freezes a live TensorFlow session (``graph_util.
convert_variables_to_constants`` + ``strip_unused``, Py/util/tf.py:50-196). There is no
TensorFlow runtime in this framework: the "session" is a :class:`zoo.tfpark.TFNet`
(a GraphDef / SavedModel / export folder executed on the MI355X), whose variables may
have been trained since loading. ``export_tf`` writes its sub-graph between ``inputs``
and ``outputs`` with every variable replaced by a ``Const`` holding the CURRENT value
and variable reads turned into ``Identity`` -- exactly the frozen form the reference
produces -- so the folder loads back with ``TFNet.from_export_folder`` here, and with
TensorFlow's own GraphDef importer elsewhere. Nodes that are kept are written back
byte-for-byte from the original GraphDef.
"""
import json
import os

import numpy as np

from zoo.utils import protobuf as pb

# numpy dtype -> TF DataType enum
_TF_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
          np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
          np.dtype(np.uint16): 17, np.dtype(np.float16): 19}
_VAR_OPS = ("VariableV2", "Variable", "VarHandleOp")


def _name(t):
    return t if isinstance(t, str) else getattr(t, "name", str(t))


def tensor_proto(arr):
    """numpy array -> serialized TensorProto (dtype, shape, tensor_content; strings / bytes ->
    DT_STRING string_val)."""
    arr = np.asarray(arr)
    if arr.dtype == object or arr.dtype.kind in ("S", "U"):
        shape = b"".join(pb.enc_bytes(2, pb.enc_int(1, int(d))) for d in arr.shape)
        vals = [v.encode() if isinstance(v, str) else bytes(v) for v in arr.reshape(-1).tolist()]
        return pb.enc_int(1, 7) + pb.enc_bytes(2, shape) + b"".join(pb.enc_bytes(8, v) for v in vals)
    arr = np.ascontiguousarray(arr)
    dt = _TF_DT.get(arr.dtype)
    if dt is None:
        raise TypeError("export_tf: unsupported dtype %s" % arr.dtype)
    shape = b"".join(pb.enc_bytes(2, pb.enc_int(1, int(d))) for d in arr.shape)
    return pb.enc_int(1, dt) + pb.enc_bytes(2, shape) + pb.enc_bytes(4, arr.astype(arr.dtype.newbyteorder("<"))
                                                                       .tobytes())


def _attr_entry(key, attr_value):
    return pb.enc_bytes(5, pb.enc_bytes(1, key.encode()) + pb.enc_bytes(2, attr_value))


def const_node(name, arr):
    arr = np.asarray(arr)
    dt = 7 if (arr.dtype == object or arr.dtype.kind in ("S", "U")) else _TF_DT[np.ascontiguousarray(arr).dtype]
    return (pb.enc_bytes(1, name.encode()) + pb.enc_bytes(2, b"Const") +
            _attr_entry("dtype", pb.enc_int(6, dt)) +
            _attr_entry("value", pb.enc_bytes(8, tensor_proto(arr))))


def identity_node(name, inp, dtype):
    return (pb.enc_bytes(1, name.encode()) + pb.enc_bytes(2, b"Identity") + pb.enc_bytes(3, inp.encode()) +
            _attr_entry("T", pb.enc_int(6, int(dtype) % 100)))


def freeze_graph(net, inputs, outputs):
    """-> (serialized GraphDef bytes, [frozen variable names]) of ``net`` (a TFNet)."""
    from zoo.pipeline.api.net.tf_graph import split_name
    graph = net._graph  # noqa: SLF001 - same package family
    values = net._values()  # noqa: SLF001
    keep = graph.needed(outputs, inputs)
    feed_nodes = {split_name(t)[0] for t in inputs}
    out, frozen = [], []
    for n in keep:
        node = graph.nodes[n]
        if node.op in _VAR_OPS:
            v = values[n].detach().float().cpu().numpy() if hasattr(values[n], "detach") else np.asarray(values[n])
            out.append(const_node(n, v.astype(np.float32) if v.dtype == np.float64 else v))
            frozen.append(n)
        elif node.op == "ReadVariableOp":
            out.append(identity_node(n, node.inputs[0], node.attr.get("dtype", 1)))
        elif n in feed_nodes and node.op != "Placeholder":
            # an input that is an interior tensor becomes a placeholder of its dtype
            dt = int(node.attr.get("T", node.attr.get("dtype", 1)))
            out.append(pb.enc_bytes(1, n.encode()) + pb.enc_bytes(2, b"Placeholder") +
                       _attr_entry("dtype", pb.enc_int(6, dt % 100)))
        else:
            if node.raw is None:
                raise ValueError("node %s has no serialized form" % n)
            # drop control inputs (initializers / savers are not exported); NodeDef fields
            # are all length-delimited, repeated fields keep their order
            if node.controls:
                g = pb.group(node.raw)
                out.append(b"".join(pb.enc_bytes(f, v) for f in sorted(g) for _w, v in g[f]
                                    if not (f == 3 and pb.as_str(v).startswith("^"))))
            else:
                out.append(node.raw)
    gd = b"".join(pb.enc_bytes(1, nd) for nd in out)
    return gd, frozen


def export_tf(sess, folder, inputs, outputs, generate_backward=False, allow_non_differentiable_input=True):
    """Freeze ``sess`` (a :class:`zoo.tfpark.TFNet`) between ``inputs`` and ``outputs``
    (tensor names, or objects with ``.name``) into ``folder``. ``generate_backward``: the
    reference also exports the gradient graph for TFTrainingHelper; here TFNet
    differentiates the frozen graph itself (torch autograd), so the flag is recorded in
    the meta only."""
    from zoo.tfpark.tfnet import TFNet
    if not isinstance(sess, TFNet):
        raise TypeError("export_tf freezes a zoo.tfpark.TFNet (there is no TensorFlow session in this framework); "
                        "got %r" % type(sess))
    inputs = [_name(t) for t in inputs]
    outputs = [_name(t) for t in outputs]
    os.makedirs(folder, exist_ok=True)
    gd, frozen = freeze_graph(sess, inputs, outputs)
    with open(os.path.join(folder, "frozen_inference_graph.pb"), "wb") as f:
        f.write(gd)
    meta = {"input_names": inputs, "output_names": outputs, "variables": [], "frozen_variables": frozen,
            "generate_backward": bool(generate_backward)}
    with open(os.path.join(folder, "graph_meta.json"), "w") as f:
        json.dump(meta, f, indent=2)
    return folder


def strip_unused(net, input_names, output_names):
    """The sub-graph of ``net`` needed for ``output_names`` given ``input_names`` (node names)."""
    return net._graph.needed(output_names, input_names)  # noqa: SLF001


def attr_value(v):
    """Python value -> serialized AttrValue (int -> i, float -> f, bool -> b, str/bytes -> s,
    ("type", dt) -> type, ("shape", dims) -> shape, np.ndarray -> tensor, list of ints -> list.i)."""
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "type":
        return pb.enc_int(6, int(v[1]))
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "func":          # NameAttrList
        return pb.enc_bytes(10, pb.enc_bytes(1, v[1].encode()))
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "types":         # list(type)
        return pb.enc_bytes(1, pb.enc_packed_ints(6, [int(t) for t in v[1]]))
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "shapes":        # list(shape)
        return pb.enc_bytes(1, b"".join(
            pb.enc_bytes(7, b"".join(pb.enc_bytes(2, pb.enc_int(1, int(d) & 0xFFFFFFFFFFFFFFFF)) for d in dims))
            for dims in v[1]))
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "strings":       # list(string)
        return pb.enc_bytes(1, b"".join(pb.enc_bytes(2, x.encode() if isinstance(x, str) else x) for x in v[1]))
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "shape":
        return pb.enc_bytes(7, b"".join(pb.enc_bytes(2, pb.enc_int(1, int(d) & 0xFFFFFFFFFFFFFFFF)) for d in v[1]))
    if isinstance(v, bool):
        return pb.enc_int(5, 1 if v else 0)
    if isinstance(v, int):
        return pb.enc_int(3, v & 0xFFFFFFFFFFFFFFFF)
    if isinstance(v, float):
        return pb.enc_float(4, v)
    if isinstance(v, (str, bytes)):
        return pb.enc_bytes(2, v.encode() if isinstance(v, str) else v)
    if isinstance(v, np.ndarray):
        return pb.enc_bytes(8, tensor_proto(v))
    if isinstance(v, (list, tuple)):
        return pb.enc_bytes(1, b"".join(pb.enc_int(3, int(x) & 0xFFFFFFFFFFFFFFFF) for x in v))
    raise TypeError("attr_value: %r" % type(v))


def node_def(name, op, inputs=(), **attrs):
    """A serialized NodeDef (programmatic TF graph building, e.g. for tests and exports)."""
    out = pb.enc_bytes(1, name.encode()) + pb.enc_bytes(2, op.encode())
    for i in inputs:
        out += pb.enc_bytes(3, i.encode())
    for k, v in attrs.items():
        out += _attr_entry(k, attr_value(v))
    return out


def graph_def(nodes, library=()):
    """Serialized GraphDef from serialized NodeDefs (+ FunctionDefs for its function library)."""
    out = b"".join(pb.enc_bytes(1, n) for n in nodes)
    if library:
        out += pb.enc_bytes(2, b"".join(pb.enc_bytes(1, f) for f in library))
    return out


def function_def(name, inputs, outputs, nodes, ret):
    """Serialized FunctionDef: ``inputs`` / ``outputs`` lists of (arg name, TF dtype enum), body
    ``nodes`` (NodeDefs whose inputs use the function naming ``arg`` / ``node:out_arg:i``) and
    ``ret`` {output arg: "node:out_arg:i"} (a tf.data map / filter function)."""
    sig = pb.enc_bytes(1, name.encode())
    for n, dt in inputs:
        sig += pb.enc_bytes(2, pb.enc_bytes(1, n.encode()) + pb.enc_int(3, int(dt)))
    for n, dt in outputs:
        sig += pb.enc_bytes(3, pb.enc_bytes(1, n.encode()) + pb.enc_int(3, int(dt)))
    out = pb.enc_bytes(1, sig) + b"".join(pb.enc_bytes(3, n) for n in nodes)
    for k, v in ret.items():
        out += pb.enc_bytes(4, pb.enc_bytes(1, k.encode()) + pb.enc_bytes(2, v.encode()))
    return out

