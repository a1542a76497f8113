"""TFNet: run a TensorFlow graph (frozen ``.pb``, ``export_tf`` folder or
SavedModel) as a layer (Py/tfpark/tfnet.py:52-300; Zs/pipeline/api/net/TFNet.scala:57-620,
TFNetForInference.scala).

The reference hands the graph to libtensorflow through JNI. Here the graph is
decoded with the safe protobuf codec and executed op by op with PyTorch-ROCm
(zoo.pipeline.api.net.tf_graph): a TFNet is an ordinary ``nn.Module`` — it
moves to ``cuda`` with ``.to()``, serves through InferenceModel, and its
backward is torch autograd through the same ops (the reference needed the
exported gradient sub-graph for that; those ``*Grad`` ops are supported too so
an exported training graph still runs as-is).

Weights: Const nodes become buffers (frozen, like the reference's inference
TFNet); SavedModel variables become parameters (``trainable=True`` lets the
engine fine-tune them).
"""
import os
import warnings

import numpy as np
import torch
import torch.nn as nn

from zoo.pipeline.api.net.tf_graph import (TFGraph, graph_meta, load_saved_model, parse_graph_def,
                                           split_name, torch_dtype)


def _buf_name(i):
    return "c%d" % i


class TFNet(nn.Module):
    def __init__(self, path=None, input_names=None, output_names=None, tf_session_config=None, tag="serve",
                 signature=None, trainable=False, _nodes=None, _variables=None):
        super().__init__()
        if isinstance(input_names, str):
            input_names = [input_names]
        if isinstance(output_names, str):
            output_names = [output_names]
        variables = _variables or {}
        if _nodes is not None:
            nodes = _nodes
        elif path is not None and os.path.isdir(path) and os.path.exists(os.path.join(path, "graph_meta.json")):
            meta = graph_meta(path)
            with open(os.path.join(path, "frozen_inference_graph.pb"), "rb") as f:
                nodes = parse_graph_def(f.read())
            input_names = input_names or meta["input_names"]
            output_names = output_names or meta["output_names"]
            self.meta = meta
        elif path is not None and os.path.isdir(path) and os.path.exists(os.path.join(path, "saved_model.pb")):
            nodes, sigs, variables = load_saved_model(path, tag)
            if input_names is None or output_names is None:
                if not sigs:
                    raise ValueError("SavedModel has no SignatureDef: pass inputs and outputs")
                sig = sigs[signature] if signature is not None else (
                    sigs.get("serving_default") or sigs[sorted(sigs)[0]])
                # the reference sorts signature inputs/outputs by key (tfnet.py:227)
                input_names = input_names or [sig["inputs"][k] for k in sorted(sig["inputs"])]
                output_names = output_names or [sig["outputs"][k] for k in sorted(sig["outputs"])]
        elif path is not None and os.path.isfile(path):
            with open(path, "rb") as f:
                nodes = parse_graph_def(f.read())
            if input_names is None or output_names is None:
                raise ValueError("a bare GraphDef needs input_names and output_names")
        else:
            raise ValueError("%s is not a TF graph file, export folder or SavedModel" % path)
        self.input_names = list(input_names)
        self.output_names = list(output_names)
        self._nodes = nodes
        self._const_names = {}
        self._host_values = {}
        self._param_names = {}
        byname = {n.name: n for n in nodes}
        self._ph_dtype = {}
        for t in self.input_names:
            n = byname.get(split_name(t)[0])
            if n is None:
                raise KeyError("input %s not in graph" % t)
            self._ph_dtype[t] = n.attr.get("dtype", 1)
        graph = TFGraph(nodes, {})
        needed = set(graph.needed(self.output_names, self.input_names))
        k = 0
        for n in nodes:
            if n.name not in needed:
                continue
            if n.op == "Const":
                v = n.attr.get("value")
                if isinstance(v, np.ndarray) and v.dtype != object:
                    t = torch.from_numpy(np.array(v, copy=True))
                    if t.is_floating_point():
                        bn = _buf_name(k)
                        k += 1
                        self.register_buffer(bn, t)
                        self._const_names[n.name] = bn
                    else:  # shapes / axes / indices stay on the host (no device round trips)
                        self._host_values[n.name] = t
                else:
                    self._host_values[n.name] = v
            elif n.op in ("VariableV2", "Variable", "VarHandleOp"):
                key = n.s("shared_name") or n.name
                if key not in variables:
                    key = n.name
                if key in variables:
                    val = torch.from_numpy(np.array(variables[key], copy=True))
                else:
                    val = self._initial_value(graph, nodes, n)
                pn = "v%d" % len(self._param_names)
                self.register_parameter(pn, nn.Parameter(val, requires_grad=bool(trainable)))
                self._param_names[n.name] = pn
        self._graph = graph

    def use_native_kernels(self, enable=True):
        """Run the graph's Conv2D / MatMul on the native MFMA kernels in bf16 (fp32 in/out) on
        the GPU; the default is exact fp32 execution with the PyTorch ops."""
        self._graph.native_bf16 = bool(enable)
        return self

    @staticmethod
    def _initial_value(graph, nodes, var):
        """A variable missing from the checkpoint takes the value of its
        initializer sub-graph (the ``Assign``/``AssignVariableOp`` feeding it),
        as ``tf.global_variables_initializer`` would."""
        for a in nodes:
            if a.op in ("Assign", "AssignVariableOp") and a.inputs and split_name(a.inputs[0])[0] == var.name:
                consts = {}
                for n in graph.needed([a.inputs[1]]):
                    nd = graph.nodes[n]
                    if nd.op == "Const":
                        v = nd.attr.get("value")
                        consts[n] = torch.from_numpy(np.array(v, copy=True)) if isinstance(v, np.ndarray) and \
                            v.dtype != object else v
                sub = TFGraph(nodes, consts)
                warnings.warn("TFNet: variable %s not in the checkpoint; using its initializer" % var.name)
                return sub.run({}, [a.inputs[1]])[0].detach().clone()
        raise KeyError("variable %s has no checkpoint value and no initializer" % var.name)

    # ------------------------------------------------------------------
    def _values(self):
        vals = dict(self._host_values)
        for n, b in self._const_names.items():
            vals[n] = getattr(self, b)
        for n, p in self._param_names.items():
            vals[n] = getattr(self, p)
        return vals

    def _device(self):
        for t in list(self.buffers()) + list(self.parameters()):
            return t.device
        return torch.device("cpu")

    def _to_input(self, x, name):
        dt = torch_dtype(self._ph_dtype.get(name, 1))
        if dt is None:  # string placeholder: numpy object array passes through
            return np.asarray(x, dtype=object)
        t = torch.as_tensor(x) if not torch.is_tensor(x) else x
        t = t.to(dt)
        return t.to(self._device()) if t.is_floating_point() else t

    def forward(self, *xs):
        if len(xs) == 1 and isinstance(xs[0], (list, tuple)):
            xs = tuple(xs[0])
        if len(xs) != len(self.input_names):
            raise ValueError("TFNet expects %d inputs (%s), got %d" % (len(self.input_names), self.input_names,
                                                                      len(xs)))
        self._graph.values = self._values()
        feeds = {n: self._to_input(x, n) for n, x in zip(self.input_names, xs)}
        outs = self._graph.run(feeds, self.output_names)
        return outs[0] if len(outs) == 1 else outs

    # ---- BigDL-style numpy API (Layer.forward / backward / predict) ----------
    def forward_numpy(self, x):
        with torch.no_grad():
            out = self.forward(*(x if isinstance(x, list) else [x]))
        return _np(out)

    def backward(self, x, grad_output):
        """d(sum(out * grad_output))/d(inputs) through torch autograd; integer
        inputs get zero gradients (TFNetSpec "work with different data types")."""
        xs = x if isinstance(x, list) else [x]
        ins = []
        for n, v in zip(self.input_names, xs):
            t = self._to_input(v, n)
            if torch.is_tensor(t) and t.is_floating_point():
                t = t.detach().requires_grad_(True)
            ins.append(t)
        with torch.enable_grad():
            outs = self.forward(*ins)
        outs = outs if isinstance(outs, list) else [outs]
        gos = grad_output if isinstance(grad_output, list) else [grad_output]
        pairs = [(o, torch.as_tensor(np.asarray(g), dtype=o.dtype, device=o.device))
                 for o, g in zip(outs, gos) if g is not None and torch.is_tensor(o) and o.requires_grad]
        diff = [t for t in ins if torch.is_tensor(t) and t.requires_grad]
        grads = torch.autograd.grad([p[0] for p in pairs], diff, [p[1] for p in pairs], allow_unused=True) \
            if pairs and diff else [None] * len(diff)
        it = iter(grads)
        res = []
        for t in ins:
            if torch.is_tensor(t) and t.requires_grad:
                g = next(it)
                res.append(np.zeros(tuple(t.shape), np.float32) if g is None else g.detach().cpu().numpy())
            else:
                res.append(np.zeros(np.shape(t), np.float32))
        return res[0] if len(res) == 1 else res

    def predict(self, x, batch_per_thread=32, distributed=False, mini_batch=False):
        xs = x if isinstance(x, list) else [x]
        n = len(xs[0])
        outs = []
        with torch.no_grad():
            for i in range(0, n, batch_per_thread):
                o = self.forward(*[a[i:i + batch_per_thread] for a in xs])
                outs.append(_np(o))
        if isinstance(outs[0], list):
            return [np.concatenate([o[k] for o in outs]) for k in range(len(outs[0]))]
        return np.concatenate(outs)

    # ---- constructors (Py/tfpark/tfnet.py:199-300) -----------------------------
    @staticmethod
    def from_export_folder(folder, tf_session_config=None):
        if not os.path.isdir(folder):
            raise ValueError(folder + " does not exist")
        return TFNet(folder)

    @staticmethod
    def from_saved_model(model_path, tag=None, signature=None, inputs=None, outputs=None,
                         tf_session_config=None, init_op=None, trainable=False):
        return TFNet(model_path, inputs, outputs, tag=tag or "serve", signature=signature, trainable=trainable)

    @staticmethod
    def from_graph_def(path, inputs, outputs):
        return TFNet(path, inputs, outputs)

    @staticmethod
    def from_session(sess, inputs, outputs, generate_backward=False, allow_non_differentiable_input=True,
                     tf_session_config=None):
        raise NotImplementedError("from_session needs a live TensorFlow session; save it with "
                                  "tf.saved_model / export_tf and use from_saved_model / from_export_folder")


def _np(o):
    if isinstance(o, list):
        return [_np(v) for v in o]
    if torch.is_tensor(o):
        return o.detach().cpu().numpy()
    return np.asarray(o)
