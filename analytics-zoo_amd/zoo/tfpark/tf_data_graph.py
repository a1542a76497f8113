"""tf.data pipelines executed from their serialized dataset graph (T4 TFDataFeatureSet,
Zs/tfpark/TFDataFeatureSet.scala:31-203; Py/tfpark/tf_dataset.py TFDataDataset).

The reference ships a ``tf.data.Dataset`` to every executor as its serialized graph
(``dataset._as_serialized_graph()``) and re-instantiates it there with TensorFlow. There is no
TensorFlow runtime in this framework, so the dataset GraphDef is interpreted directly:

* dataset ops -- TensorSliceDataset / TensorDataset / RangeDataset / TFRecordDataset (native
  TFRecord framing), MapDataset / ParallelMapDataset(V2), FilterDataset, BatchDataset(V2),
  UnbatchDataset, Shuffle(V2/V3) / ShuffleAndRepeat, Repeat, Take, Skip, Zip, Concatenate and
  the pass-through Prefetch / Model / Optimize / Cache / thread-pool wrappers -- become Python
  iterators over element tuples (numpy);
* map / filter functions are FunctionDefs of the graph's library, run on the graph executor
  (zoo.pipeline.api.net.tf_graph.TFGraph, the same one TFNet uses) with their function-style
  input names (``arg``, ``node:out_arg:i``) rewritten to graph tensor names; the tf.Example
  parsers (ParseExampleV2 / ParseSingleExample, dense features) are added to its op table.

``TFDataGraph(graph_bytes).elements()`` yields element tuples; ``TFDataset.from_tf_data_dataset``
accepts such a graph (bytes, a path, or an object with ``_as_serialized_graph``) and feeds the
unbatched elements to the native FeatureSet.
"""
import numpy as np
import torch

from zoo.pipeline.api.net import tf_graph as TG
from zoo.utils import protobuf as pb

_PASS = {"PrefetchDataset", "ModelDataset", "OptimizeDataset", "OptimizeDatasetV2", "MaxIntraOpParallelismDataset",
         "PrivateThreadPoolDataset", "CacheDataset", "CacheDatasetV2", "ExperimentalMaxIntraOpParallelismDataset",
         "ExperimentalPrivateThreadPoolDataset", "AssertCardinalityDataset", "OptionsDataset"}
_BATCH = {"BatchDataset", "BatchDatasetV2"}


# ----------------------------------------------------------------------------- FunctionDef
class _Function:
    def __init__(self, b):
        g = pb.group(b)
        sig = pb.group(g[1][0][1])
        self.name = pb.as_str(sig[1][0][1])
        self.inputs = [pb.as_str(pb.group(v)[1][0][1]) for _w, v in sig.get(2, [])]
        self.outputs = [pb.as_str(pb.group(v)[1][0][1]) for _w, v in sig.get(3, [])]
        self.nodes = [TG.parse_node(v) for _w, v in g.get(3, [])]
        self.ret = {}
        for _w, v in g.get(4, []):
            e = pb.group(v)
            self.ret[pb.as_str(e[1][0][1])] = pb.as_str(e[2][0][1])
        by_name = {n.name: n for n in self.nodes}
        for n in self.nodes:
            n.inputs = [_graph_name(t, by_name) for t in n.inputs]
            n.controls = [c for c in n.controls if c in by_name]
        self.fetches = [_graph_name(self.ret[o], by_name) for o in self.outputs]
        values = {}
        for n in self.nodes:
            if n.op == "Const":
                v = n.attr.get("value")
                values[n.name] = torch.from_numpy(np.array(v, copy=True)) if isinstance(v, np.ndarray) and \
                    v.dtype != object else v
        self.graph = TG.TFGraph(self.nodes, values)

    def __call__(self, *args):
        if len(args) != len(self.inputs):
            raise ValueError("function %s takes %d arguments, got %d" % (self.name, len(self.inputs), len(args)))
        feeds = {a: _to_graph_value(v) for a, v in zip(self.inputs, args)}
        return tuple(_to_numpy(v) for v in self.graph.run(feeds, self.fetches))


def _multi_out_index(node, out_arg, i):
    """Flat output index of ``node``'s output ``out_arg:i`` (function-body naming)."""
    op, a = node.op, node.attr
    if op in ("ParseExampleV2", "ParseSingleExample"):
        ns = int(a.get("num_sparse", 0) or 0)
        nd = len(a.get("Tdense") or [])
        order = [("sparse_indices", ns), ("sparse_values", ns), ("sparse_shapes", ns), ("dense_values", nd)]
        base = 0
        for nm, cnt in order:
            if nm == out_arg:
                return base + i
            base += cnt
        raise NotImplementedError("%s output %s" % (op, out_arg))
    return i


def _graph_name(t, by_name):
    parts = t.split(":")
    if len(parts) == 1:
        return t                       # a function argument (fed) or a node's first output
    if len(parts) == 2:
        return t
    node, out_arg, i = parts[0], parts[1], int(parts[2])
    n = by_name.get(node)
    return "%s:%d" % (node, _multi_out_index(n, out_arg, i) if n is not None else i)


def _to_graph_value(v):
    v = np.asarray(v)
    if v.dtype == object or v.dtype.kind in ("S", "U"):
        return v
    return torch.from_numpy(np.array(v, copy=True))


def _to_numpy(v):
    if torch.is_tensor(v):
        return v.detach().cpu().numpy()
    return np.asarray(v)


# ----------------------------------------------------------------------------- Example parsing
def _example_values(rec, key, dtype, shape, default):
    from zoo.tfpark.tf_dataset import parse_example
    ex = parse_example(bytes(rec))
    k = key.decode() if isinstance(key, (bytes, bytearray)) else str(key)
    if k in ex:
        v = np.asarray(ex[k])
    elif default is not None and np.asarray(default).size:
        v = np.asarray(default)
    else:
        raise KeyError("feature %s missing and no default" % k)
    npd = TG.DTYPES.get(int(dtype), np.float32)
    if npd is not object:
        v = v.astype(npd)
    if shape is None or -1 in list(shape):
        return v
    return v.reshape(list(shape))           # [] -> a scalar feature


def _parse_dense(serialized, keys, tdense, shapes, defaults):
    ser = np.asarray(serialized, dtype=object)
    recs = ser.reshape(-1)
    outs = []
    for j, key in enumerate(keys):
        d = None if j >= len(defaults) else _to_numpy(defaults[j]) if defaults[j] is not None else None
        vals = [_example_values(r, key, tdense[j], shapes[j] if j < len(shapes) else None, d) for r in recs]
        arr = np.stack(vals) if ser.ndim else vals[0]
        outs.append(_to_graph_value(arr))
    return outs


def _parse_example_v2(g, node, serialized, names, sparse_keys, dense_keys, ragged_keys, *dense_defaults):
    if int(node.attr.get("num_sparse", 0) or 0) or np.asarray(ragged_keys).size:
        raise NotImplementedError("ParseExampleV2: only dense features are supported")
    keys = list(np.asarray(dense_keys, dtype=object).reshape(-1))
    return _parse_dense(serialized, keys, node.attr.get("Tdense") or [], node.attr.get("dense_shapes") or [],
                        list(dense_defaults))


def _parse_single_example(g, node, serialized, *dense_defaults):
    if int(node.attr.get("num_sparse", 0) or 0):
        raise NotImplementedError("ParseSingleExample: only dense features are supported")
    keys = node.attr.get("dense_keys") or []
    return _parse_dense(np.asarray(serialized, dtype=object).reshape(()), keys, node.attr.get("Tdense") or [],
                        node.attr.get("dense_shapes") or [], list(dense_defaults))


def _decode_raw(g, node, x):
    npd = TG.DTYPES.get(int(node.attr.get("out_type", 1)), np.float32)
    arr = np.asarray(x, dtype=object)
    rows = [np.frombuffer(bytes(r), dtype=npd) for r in arr.reshape(-1)]
    out = np.stack(rows).reshape(arr.shape + (-1,)) if arr.ndim else rows[0]
    return _to_graph_value(out)


TG._OPS.setdefault("ParseExampleV2", _parse_example_v2)
TG._OPS.setdefault("ParseSingleExample", _parse_single_example)
TG._OPS.setdefault("DecodeRaw", _decode_raw)


# ----------------------------------------------------------------------------- dataset graph
class TFDataGraph:
    """A serialized tf.data dataset graph, iterable without TensorFlow."""

    def __init__(self, graph, output=None, seed=0):
        if isinstance(graph, str):
            with open(graph, "rb") as f:
                graph = f.read()
        g = pb.group(graph)
        self.nodes = {n.name: n for n in (TG.parse_node(v) for _w, v in g.get(1, []))}
        self.functions = {}
        for _w, lib in g.get(2, []):
            for _w2, fb in pb.group(lib).get(1, []):
                f = _Function(fb)
                self.functions[f.name] = f
        values = {}
        for n in self.nodes.values():
            if n.op == "Const":
                v = n.attr.get("value")
                values[n.name] = torch.from_numpy(np.array(v, copy=True)) if isinstance(v, np.ndarray) and \
                    v.dtype != object else v
        self._consts = TG.TFGraph(list(self.nodes.values()), values)
        self.output = output or self._find_output()
        self.seed = seed

    def _find_output(self):
        for n in self.nodes.values():
            if n.op in ("_Retval", "Identity") and n.inputs and self._is_dataset(TG.split_name(n.inputs[0])[0]):
                return TG.split_name(n.inputs[0])[0]
        used = {TG.split_name(i)[0] for n in self.nodes.values() for i in n.inputs}
        cands = [n.name for n in self.nodes.values() if n.op.endswith("Dataset") or "Dataset" in n.op]
        outs = [c for c in cands if c not in used]
        if len(outs) != 1:
            raise ValueError("cannot tell the output dataset of the graph (candidates: %s); pass output=" % outs)
        return outs[0]

    def _is_dataset(self, name):
        n = self.nodes.get(name)
        return n is not None and "Dataset" in n.op

    def _value(self, t):
        v = self._consts.run({}, [t])[0]
        return _to_numpy(v)

    def _fn(self, node, key):
        f = node.attr.get(key)
        name = f["func"] if isinstance(f, dict) else f
        if name not in self.functions:
            raise KeyError("function %s not in the graph library" % name)
        return self.functions[name]

    # ------------------------------------------------------------------ iterators
    def _it(self, name):
        node = self.nodes[name]
        op = node.op
        ins = node.inputs
        if op in _PASS:
            return self._it(TG.split_name(ins[0])[0])
        if op == "TensorSliceDataset":
            comps = [self._value(t) for t in ins]
            n = len(comps[0])
            return (tuple(c[i] for c in comps) for i in range(n))
        if op == "TensorDataset":
            comps = tuple(self._value(t) for t in ins)
            return iter([comps])
        if op == "RangeDataset":
            a, b, c = (int(self._value(t)) for t in ins[:3])
            return ((np.int64(i),) for i in range(a, b, c))
        if op in ("TFRecordDataset", "TFRecordDatasetV2"):
            from zoo.tfpark.tf_dataset import read_tfrecord
            files = [f.decode() if isinstance(f, (bytes, bytearray)) else str(f)
                     for f in np.asarray(self._value(ins[0]), dtype=object).reshape(-1)]
            return ((np.asarray(rec, dtype=object),) for fpath in files for rec in read_tfrecord(fpath))
        if op in ("MapDataset", "ParallelMapDataset", "ParallelMapDatasetV2"):
            src = self._it(TG.split_name(ins[0])[0])
            n_extra = len(node.attr.get("Targuments") or [])
            extra = tuple(self._value(t) for t in ins[1:1 + n_extra])
            f = self._fn(node, "f")
            return (f(*(tuple(e) + extra)) for e in src)
        if op == "FilterDataset":
            src = self._it(TG.split_name(ins[0])[0])
            extra = tuple(self._value(t) for t in ins[1:])
            f = self._fn(node, "predicate")
            return (e for e in src if bool(np.asarray(f(*(tuple(e) + extra))[0])))
        if op in _BATCH:
            src = self._it(TG.split_name(ins[0])[0])
            bs = int(self._value(ins[1]))
            drop = bool(self._value(ins[2])) if op == "BatchDatasetV2" and len(ins) > 2 else False
            return self._batch(src, bs, drop)
        if op == "UnbatchDataset":
            src = self._it(TG.split_name(ins[0])[0])
            return (tuple(c[i] for c in e) for e in src for i in range(len(e[0])))
        if op in ("ShuffleDataset", "ShuffleDatasetV2", "ShuffleDatasetV3", "ShuffleAndRepeatDataset"):
            buf = int(self._value(ins[1]))
            seed = self.seed
            if op in ("ShuffleDataset", "ShuffleDatasetV3", "ShuffleAndRepeatDataset") and len(ins) > 3:
                seed = (int(self._value(ins[2])) * 1000003 + int(self._value(ins[3]))) or self.seed
            count = int(self._value(ins[4])) if op == "ShuffleAndRepeatDataset" else 1
            return self._shuffle(TG.split_name(ins[0])[0], buf, seed, count)
        if op == "RepeatDataset":
            return self._repeat(TG.split_name(ins[0])[0], int(self._value(ins[1])))
        if op == "TakeDataset":
            src = self._it(TG.split_name(ins[0])[0])
            k = int(self._value(ins[1]))
            return src if k < 0 else _take(src, k)
        if op == "SkipDataset":
            src = self._it(TG.split_name(ins[0])[0])
            k = int(self._value(ins[1]))
            return (e for i, e in enumerate(src) if i >= k)
        if op == "ZipDataset":
            its = [self._it(TG.split_name(t)[0]) for t in ins]
            return (tuple(c for e in es for c in e) for es in zip(*its))
        if op == "ConcatenateDataset":
            a, b = (self._it(TG.split_name(t)[0]) for t in ins[:2])
            return (e for it in (a, b) for e in it)
        raise NotImplementedError("tf.data op %s (node %s) is not supported" % (op, name))

    @staticmethod
    def _batch(src, bs, drop):
        buf = []
        for e in src:
            buf.append(e)
            if len(buf) == bs:
                yield tuple(np.stack([x[i] for x in buf]) for i in range(len(buf[0])))
                buf = []
        if buf and not drop:
            yield tuple(np.stack([x[i] for x in buf]) for i in range(len(buf[0])))

    def _shuffle(self, name, buf_size, seed, count):
        rng = np.random.RandomState(seed & 0x7FFFFFFF)
        for _ in (range(count) if count >= 0 else iter(int, 1)):
            buf = []
            for e in self._it(name):
                buf.append(e)
                if len(buf) >= buf_size:
                    yield buf.pop(rng.randint(len(buf)))
            while buf:
                yield buf.pop(rng.randint(len(buf)))

    def _repeat(self, name, count):
        k = 0
        while count < 0 or k < count:
            for e in self._it(name):
                yield e
            k += 1

    def elements(self):
        """Iterator over the dataset's element tuples (numpy arrays)."""
        return self._it(self.output)

    def unbatched(self):
        """Element tuples with a trailing Batch op undone (the FeatureSet batches itself)."""
        node = self.nodes[self.output]
        name = self.output
        while node.op in _PASS:
            name = TG.split_name(node.inputs[0])[0]
            node = self.nodes[name]
        if node.op in _BATCH:
            return self._it(TG.split_name(node.inputs[0])[0])
        return self.elements()


def _take(src, k):
    for i, e in enumerate(src):
        if i >= k:
            return
        yield e


def serialized_graph(dataset):
    """GraphDef bytes of ``dataset``: bytes / a path / an object with ``_as_serialized_graph``
    (a tf.data.Dataset), else None."""
    if isinstance(dataset, (bytes, bytearray)):
        return bytes(dataset)
    if isinstance(dataset, str):
        with open(dataset, "rb") as f:
            return f.read()
    fn = getattr(dataset, "_as_serialized_graph", None)
    if fn is not None:
        g = fn()
        return g.numpy() if hasattr(g, "numpy") else bytes(g)
    return None


__all__ = ["TFDataGraph", "serialized_graph"]
