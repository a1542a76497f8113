"""KerasNet / Model / Sequential / Merge.

Parity: Py/pipeline/api/keras/engine/topology.py:31-406 and
Zs/pipeline/api/keras/models/Topology.scala (KerasNet 65-602, Model 604-706,
Sequential 827-960): compile (objects or strings), fit (ndarrays, FeatureSet,
ImageSet, TextSet, DataLoader; distributed or local), evaluate, predict,
predict_classes, summary, TensorBoard summaries, checkpointing, constant /
L2-norm gradient clipping, save/load, get_layer, freeze.

Training runs on :class:`zoo.pipeline.engine.TrainingEngine` (one process per
GPU, RCCL gradient sync) — the replacement of InternalDistriOptimizer.
"""
import logging
import os

import numpy as np
import torch
import torch.nn as nn

from zoo.pipeline.api.keras.base import Input, InputLayer, Layer, Node, Variable, _flatten_vars, is_symbolic, \
    to_shape

log = logging.getLogger("zoo.keras")


def _to_tensor(a):
    if isinstance(a, torch.Tensor):
        return a
    if isinstance(a, (list, tuple)):
        return [_to_tensor(e) for e in a]
    arr = np.asarray(a)
    if arr.dtype == np.float64:
        arr = arr.astype(np.float32)
    return torch.from_numpy(np.ascontiguousarray(arr))


def _to_numpy(t):
    if isinstance(t, (list, tuple)):
        return [_to_numpy(e) for e in t]
    return t.detach().float().cpu().numpy() if t.is_floating_point() else t.detach().cpu().numpy()


class KerasNet(Layer):
    """Base of trainable containers."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._criterion = None
        self._optim = None
        self._metrics = []
        self._engine = None
        self._tb = None
        self._ckpt = None
        self._clip = None

    # ------------------------------------------------------------------ compile
    def compile(self, optimizer, loss, metrics=None):
        from zoo.pipeline.api.keras.metrics import to_metrics
        from zoo.pipeline.api.keras.objectives import to_criterion
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        self._optim = to_optim_method(optimizer)
        self._criterion = to_criterion(loss)
        self._metrics = to_metrics(metrics, self._criterion)
        self._engine = None
        return self

    def _loss_fn(self):
        crit = self._criterion
        regs = [m for m in self.modules() if isinstance(m, Layer) and m._regularizers]

        def f(out, target):
            l = crit(out, target)
            for m in regs:
                l = l + m.regularization_loss()
            return l
        return f

    def _get_engine(self):
        if self._engine is None:
            if self._criterion is None:
                raise RuntimeError("call compile() before fit()")
            from zoo.pipeline.engine import TrainingEngine
            self._engine = TrainingEngine(self, self._loss_fn(), self._optim, clip=self._clip)
            if self._tb is not None:
                self._engine.train_summary, self._engine.val_summary = self._tb
            if self._ckpt is not None:
                self._engine.set_checkpoint(*self._ckpt)
        return self._engine

    # ------------------------------------------------------------------ config
    def set_tensorboard(self, log_dir, app_name):
        from zoo.tensorboard import TrainSummary, ValidationSummary
        self._tb = (TrainSummary(log_dir, app_name), ValidationSummary(log_dir, app_name))
        if self._engine is not None:
            self._engine.train_summary, self._engine.val_summary = self._tb

    def get_train_summary(self, tag=None):
        if self._tb is None:
            return None
        return self._tb[0].read_scalar(tag or "Loss")

    def get_validation_summary(self, tag=None):
        if self._tb is None:
            return None
        return self._tb[1].read_scalar(tag)

    def set_checkpoint(self, path, over_write=True):
        from zoo.common.triggers import EveryEpoch
        self._ckpt = (path, EveryEpoch(), over_write)
        if self._engine is not None:
            self._engine.set_checkpoint(*self._ckpt)

    def clear_gradient_clipping(self):
        self._clip = None
        if self._engine is not None:
            self._engine.clip = None

    def set_constant_gradient_clipping(self, min, max):  # noqa: A002
        from zoo.parallel.ddp import constant_clip
        self._clip = constant_clip(float(min), float(max))
        if self._engine is not None:
            self._engine.clip = self._clip

    def set_gradient_clipping_by_l2_norm(self, clip_norm):
        from zoo.parallel.ddp import global_norm_clip
        self._clip = global_norm_clip(float(clip_norm))
        if self._engine is not None:
            self._engine.clip = self._clip

    def set_evaluate_status(self):
        self.eval()
        return self

    # ------------------------------------------------------------------ data
    def _make_featureset(self, x, y, batch_size, shuffle=True):
        from zoo.feature.common import FeatureSet
        if hasattr(x, "to_featureset"):
            x = x.to_featureset(batch_size)
        if isinstance(x, FeatureSet):
            return x
        if isinstance(x, torch.utils.data.DataLoader):
            return FeatureSet.from_dataloader(x)
        return FeatureSet.from_ndarrays(_to_tensor(x), None if y is None else _to_tensor(y), batch_size,
                                        shuffle=shuffle)

    # ------------------------------------------------------------------ fit
    def fit(self, x, y=None, batch_size=32, nb_epoch=10, validation_data=None, distributed=True,
            validation_trigger=None):
        from zoo.common.triggers import MaxEpoch
        eng = self._get_engine()
        data = self._make_featureset(x, y, batch_size, shuffle=True)
        val = None
        if validation_data is not None:
            if isinstance(validation_data, (list, tuple)) and len(validation_data) == 2:
                val = self._make_featureset(validation_data[0], validation_data[1], batch_size, shuffle=False)
            else:
                val = self._make_featureset(validation_data, None, batch_size, shuffle=False)
        start_epoch = eng.state["epoch"]
        eng.fit(data, end_trigger=MaxEpoch(start_epoch + nb_epoch - 1), validation=val,
                val_methods=self._metrics if val is not None else None, val_trigger=validation_trigger)
        return self

    def get_finished_epoch(self):
        return self._engine.state["epoch"] - 1 if self._engine else 0

    # ------------------------------------------------------------------ eval
    def evaluate(self, x, y=None, batch_size=32):
        eng = self._get_engine()
        data = self._make_featureset(x, y, batch_size, shuffle=False)
        from zoo.pipeline.api.keras.metrics import Loss
        methods = self._metrics or [Loss(self._criterion)]
        return [v for _, v in eng.evaluate(data, methods)]

    # ------------------------------------------------------------------ predict
    @torch.no_grad()
    def predict(self, x, batch_per_thread=4, distributed=True, batch_size=None):
        from zoo.feature.common import FeatureSet
        from zoo.common.nncontext import get_nncontext
        dev = get_nncontext().device
        self.to(dev)
        was = self.training
        self.eval()
        if isinstance(x, FeatureSet) or hasattr(x, "to_featureset"):
            fs = x if isinstance(x, FeatureSet) else x.to_featureset(batch_size or 32)
            outs = []
            for b in fs.data(train=False):
                inp = b[0] if isinstance(b, (list, tuple)) else b
                outs.append(self._forward_any(inp, dev))
        else:
            xt = _to_tensor(x)
            n = (xt[0] if isinstance(xt, list) else xt).shape[0]
            bs = batch_size or max(batch_per_thread * 64, 256)
            outs = []
            for s in range(0, n, bs):
                chunk = [t[s:s + bs] for t in xt] if isinstance(xt, list) else xt[s:s + bs]
                outs.append(self._forward_any(chunk, dev))
        self.train(was)
        if not outs:
            return np.zeros((0,))
        if isinstance(outs[0], list):
            return [np.concatenate([o[i] for o in outs]) for i in range(len(outs[0]))]
        return np.concatenate(outs)

    def _forward_any(self, inp, dev):
        inp = [t.to(dev) for t in inp] if isinstance(inp, list) else inp.to(dev)
        out = self(inp) if not isinstance(inp, list) else self(*inp) if not self._wants_list() else self(inp)
        return _to_numpy(out)

    def _wants_list(self):
        return True

    def predict_classes(self, x, batch_per_thread=4, zero_based_label=True):
        p = self.predict(x, batch_per_thread)
        c = np.argmax(p, axis=-1)
        return c if zero_based_label else c + 1

    def forward_numpy(self, x):
        return self.predict(x)

    # ------------------------------------------------------------------ misc
    def save_to_keras2(self, json_path=None, hdf5_path=None):
        """KerasNet.saveToKeras2: Keras 2 definition json and/or full-model HDF5 file
        (zoo.pipeline.api.keras.keras_import.save_keras2)."""
        from zoo.pipeline.api.keras.keras_import import save_keras2
        return save_keras2(self, json_path, hdf5_path)

    saveToKeras2 = save_to_keras2

    def get_layer(self, name):
        for m in self.modules():
            if isinstance(m, Layer) and m.name == name:
                return m
        raise ValueError("No layer named %s" % name)

    @property
    def layers(self):
        return self._layer_list()

    def _layer_list(self):
        return [m for m in self.children() if isinstance(m, Layer)]

    def flattened_layers(self, include_container=False):
        out = []
        for l in self._layer_list():
            if isinstance(l, KerasNet):
                if include_container:
                    out.append(l)
                out.extend(l.flattened_layers(include_container))
            else:
                out.append(l)
        return out

    def summary(self, line_length=120, positions=(.33, .55, .67, 1.)):
        rows = [("Layer (type)", "Output Shape", "Param #")]
        total = 0
        for l in self.flattened_layers():
            n = sum(p.numel() for p in l.parameters())
            total += n
            rows.append(("%s (%s)" % (l.name, type(l).__name__), str(l.get_output_shape()), str(n)))
        w = [int(line_length * p) for p in positions]
        lines = ["_" * line_length]
        for r in rows:
            s = r[0].ljust(w[0]) + r[1].ljust(w[1] - w[0]) + r[2]
            lines.append(s)
            lines.append("=" * line_length if r is rows[0] else "_" * line_length)
        lines.append("Total params: %d" % total)
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        lines.append("Trainable params: %d" % trainable)
        lines.append("Non-trainable params: %d" % (total - trainable))
        txt = "\n".join(lines)
        print(txt)
        return txt

    def get_weights(self):
        return [w for l in self.flattened_layers() for w in l.get_weights()]

    def set_weights(self, weights):
        i = 0
        for l in self.flattened_layers():
            n = len(l.get_weights())
            if n:
                l.set_weights(weights[i:i + n])
                i += n

    def save(self, path, over_write=False):
        from zoo.pipeline.api.keras.serialization import save_model
        save_model(self, path, over_write)

    def save_model(self, path, weight_path=None, over_write=False):
        self.save(path, over_write)

    def freeze_up_to(self, names):
        names = [names] if isinstance(names, str) else names
        for l in self.flattened_layers():
            l.freeze()
            if l.name in names:
                break
        return self

    def unfreeze(self, names=None):
        for l in self.flattened_layers():
            if names is None or l.name in names:
                l.unfreeze()
        return self

    def to_model(self):
        return self


class Sequential(KerasNet):
    """Linear stack of layers (models.py:29, Topology.scala:827-960)."""

    def __init__(self, name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.stack = nn.ModuleList()

    def is_built(self):
        return len(self.stack) > 0 and self._output_shape is not None

    def add(self, layer):
        if len(self.stack) == 0:
            shape = layer._given_input_shape if not isinstance(layer, KerasNet) else \
                (layer.get_input_shape()[1:] if layer.get_input_shape() else None)
            if shape is None:
                raise ValueError("The first layer of a Sequential model needs input_shape")
            in_shape = (None,) + to_shape(shape) if not isinstance(shape, list) else shape
            self._input_shape = in_shape
            cur = in_shape
        else:
            cur = self._output_shape
        if isinstance(layer, InputLayer):
            self._output_shape = cur
            return self
        layer._ensure_built(cur)
        self._output_shape = layer.compute_output_shape(cur)
        layer._output_shape = self._output_shape
        self.stack.append(layer)
        self.built = True
        return self

    def compute_output_shape(self, input_shape):
        return self._output_shape

    def build(self, input_shape):
        pass

    def call(self, x):
        for l in self.stack:
            x = l(x)
        return x

    def _layer_list(self):
        return list(self.stack)

    def _wants_list(self):
        return True


class Model(KerasNet):
    """Functional graph model: ``Model(input, output)`` (models.py:76, Topology.scala:604-706)."""

    def __init__(self, input, output, name=None, **kwargs):  # noqa: A002 - reference name
        super().__init__(name=name, **kwargs)
        self.inputs = list(input) if isinstance(input, (list, tuple)) else [input]
        self.outputs = list(output) if isinstance(output, (list, tuple)) else [output]
        self._multi_out = isinstance(output, (list, tuple))
        order, seen = [], set()

        def visit(v):
            node = v.node
            if id(node) in seen:
                return
            for i in node.inputs:
                visit(i)
            seen.add(id(node))
            order.append(node)
        for o in self.outputs:
            visit(o)
        self._nodes = order
        self._input_nodes = {id(v.node) for v in self.inputs}
        mods, mseen = [], set()
        for n in order:
            if id(n.layer) not in mseen and not isinstance(n.layer, InputLayer):
                mseen.add(id(n.layer))
                mods.append(n.layer)
        self.graph_layers = nn.ModuleList(mods)
        self._input_shape = [v.shape for v in self.inputs] if len(self.inputs) > 1 else self.inputs[0].shape
        self._output_shape = [v.shape for v in self.outputs] if self._multi_out else self.outputs[0].shape
        self.built = True

    def compute_output_shape(self, input_shape):
        return self._output_shape

    def call(self, x):
        xs = x if isinstance(x, (list, tuple)) else [x]
        if len(xs) != len(self.inputs):
            raise ValueError("model expects %d inputs, got %d" % (len(self.inputs), len(xs)))
        vals = {}
        for v, t in zip(self.inputs, xs):
            vals[(id(v.node), v.index)] = t
        for node in self._nodes:
            if id(node) in self._input_nodes:
                continue
            if not node.inputs:
                out = node.layer.call(None)
            else:
                args = [vals[(id(i.node), i.index)] for i in node.inputs]
                arg = args if (len(args) > 1 or getattr(node, "list_input", False)) else args[0]
                out = node.layer(arg)
            if isinstance(out, (list, tuple)) and len(node.outputs) > 1:
                for i, o in enumerate(out):
                    vals[(id(node), i)] = o
            else:
                vals[(id(node), 0)] = out
        outs = [vals[(id(v.node), v.index)] for v in self.outputs]
        return outs if self._multi_out else outs[0]

    def forward(self, x, *rest):
        if rest:
            x = [x] + list(rest)
        return self.call(x)

    def _layer_list(self):
        return list(self.graph_layers)

    def new_graph(self, outputs):
        """Sub-graph ending at the named layers' outputs (NetUtils.newGraph)."""
        names = [outputs] if isinstance(outputs, str) else outputs
        outs = []
        for n in self._nodes:
            if n.layer.name in names:
                outs.append(n.outputs[0])
        return Model(self.inputs if len(self.inputs) > 1 else self.inputs[0], outs if len(outs) > 1 else outs[0])

    def save_graph_topology(self, log_path, backward=False):
        os.makedirs(log_path, exist_ok=True)
        with open(os.path.join(log_path, "graph.txt"), "w") as f:
            for n in self._nodes:
                f.write("%s <- %s\n" % (n.layer.name, [i.node.layer.name for i in n.inputs]))


class Merge(Layer):
    """Merge a list of inputs: sum, mul, concat, ave, cos, dot, max, min (Merge.scala:235)."""

    def __init__(self, layers=None, mode="sum", concat_axis=-1, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.mode = mode.lower()
        self.concat_axis = concat_axis
        self.merge_layers = layers

    def compute_output_shape(self, input_shape):
        shapes = input_shape
        if self.mode == "concat":
            ax = self.concat_axis if self.concat_axis >= 0 else len(shapes[0]) + self.concat_axis
            out = list(shapes[0])
            out[ax] = sum(s[ax] for s in shapes)
            return tuple(out)
        if self.mode in ("cos", "dot"):
            return (None, 1)
        return shapes[0]

    def call(self, xs):
        m = self.mode
        if m == "sum":
            out = xs[0]
            for t in xs[1:]:
                out = out + t
            return out
        if m == "mul":
            out = xs[0]
            for t in xs[1:]:
                out = out * t
            return out
        if m == "ave":
            return sum(xs) / len(xs)
        if m == "max":
            out = xs[0]
            for t in xs[1:]:
                out = torch.maximum(out, t)
            return out
        if m == "min":
            out = xs[0]
            for t in xs[1:]:
                out = torch.minimum(out, t)
            return out
        if m == "concat":
            return torch.cat(xs, dim=self.concat_axis)
        if m == "dot":
            from zoo.ops.reduce import reduce   # native row reduction on the GPU (HK14)
            return reduce(xs[0] * xs[1], -1, "sum", keepdim=True)
        if m == "cos":
            from zoo.ops.reduce import l2_normalize, reduce
            a, b = l2_normalize(xs[0], -1, 1e-16), l2_normalize(xs[1], -1, 1e-16)
            return reduce(a * b, -1, "sum", keepdim=True)
        raise ValueError("Unsupported merge mode %s" % m)


def merge(inputs, mode="sum", concat_axis=-1, name=None):
    return Merge(mode=mode, concat_axis=concat_axis, name=name)(list(inputs))
