"""Keras model persistence (KerasNet.saveModel / Net.load, Topology.scala:708-825).

``save_model`` writes the reference's BigDL/Zoo ``.model`` protobuf by default
(zoo.utils.bigdl_model); ``load_model`` reads both that and the framework's
torch-file format below.

A torch-file model is ONE file written with ``torch.save`` that contains only
primitives and tensors, so it is loaded back with ``torch.load(weights_only=True)``
(nothing in the file is executed):

  {"format": "zoo-keras-v1", "arch": <config tree>, "state": <state_dict>}

The config tree records every layer's class (module + qualname) and the
constructor arguments captured by ``Layer.__init_subclass__``; nested layers
(TimeDistributed(Dense), Sequential inside Model, ...) are encoded recursively,
and functional graphs are encoded as their node list. Only classes under the
``zoo.`` package are ever instantiated on load. The BigDL ``.model`` protobuf
format of the reference is handled separately by zoo.utils.bigdl_proto.
"""
import importlib

import numpy as np
import torch

from zoo.pipeline.api.keras.base import Input, InputLayer, Layer, Variable

FORMAT = "zoo-keras-v1"


def _enc(v):
    if isinstance(v, Layer):
        return {"__layer__": layer_config(v)}
    if isinstance(v, (list, tuple)):
        return {"__seq__": [_enc(e) for e in v], "tuple": isinstance(v, tuple)}
    if isinstance(v, dict):
        return {"__dict__": {str(k): _enc(e) for k, e in v.items()}}
    if isinstance(v, np.ndarray):
        return {"__tensor__": torch.from_numpy(v.copy())}
    if isinstance(v, torch.Tensor):
        return {"__tensor__": v.detach().cpu()}
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    if hasattr(v, "l1") and hasattr(v, "l2"):  # Regularizer
        return {"__reg__": [v.l1, v.l2]}
    raise TypeError("cannot serialize constructor argument of type %s" % type(v).__name__)


def _dec(v):
    if isinstance(v, dict):
        if "__layer__" in v:
            return build_layer(v["__layer__"])
        if "__seq__" in v:
            s = [_dec(e) for e in v["__seq__"]]
            return tuple(s) if v.get("tuple") else s
        if "__dict__" in v:
            return {k: _dec(e) for k, e in v["__dict__"].items()}
        if "__tensor__" in v:
            return v["__tensor__"].numpy()
        if "__reg__" in v:
            from zoo.pipeline.api.keras.base import Regularizer
            return Regularizer(*v["__reg__"])
    return v


def _class_path(cls):
    return cls.__module__, cls.__qualname__


def _resolve(mod, qual):
    if not mod.startswith("zoo."):
        raise ValueError("refusing to instantiate non-zoo class %s.%s" % (mod, qual))
    obj = importlib.import_module(mod)
    for part in qual.split("."):
        obj = getattr(obj, part)
    if not (isinstance(obj, type) and issubclass(obj, Layer)):
        raise ValueError("%s.%s is not a zoo Layer" % (mod, qual))
    return obj


def layer_config(layer):
    from zoo.pipeline.api.keras.engine.topology import Model, Sequential
    mod, qual = _class_path(type(layer))
    if isinstance(layer, Sequential):
        return {"class": [mod, qual], "name": layer.name, "sequential": [layer_config(l) for l in layer.stack],
                "input_shape": list(layer.get_input_shape()[1:]) if layer.get_input_shape() else None}
    if isinstance(layer, Model) and type(layer).__name__ == "Model":
        return {"class": [mod, qual], "name": layer.name, "graph": graph_config(layer)}
    if not hasattr(layer, "_init_args"):
        raise TypeError("layer %s has no recorded constructor arguments" % layer.name)
    _cls, a, k = layer._init_args
    k = dict(k)
    k.setdefault("name", layer.name)
    gis = layer._given_input_shape
    return {"class": [mod, qual], "args": [_enc(x) for x in a], "kwargs": {kk: _enc(vv) for kk, vv in k.items()},
            "given_input_shape": None if gis is None else _enc(list(gis)) if not isinstance(gis, list) else _enc(gis),
            "built_shape": _enc(list(layer.get_input_shape())) if isinstance(layer.get_input_shape(), tuple) else None}


def graph_config(model):
    layers, lid = [], {}
    nodes = []
    for n in model._nodes:
        if isinstance(n.layer, InputLayer):
            shape = list(n.output_shapes[0][1:])
            nodes.append({"input": True, "shape": shape, "name": n.layer.name})
            continue
        if id(n.layer) not in lid:
            lid[id(n.layer)] = len(layers)
            layers.append(layer_config(n.layer))
        nodes.append({"layer": lid[id(n.layer)], "inbound": [[model._nodes.index(i.node), i.index] for i in n.inputs],
                      "list_input": bool(getattr(n, "list_input", False))})
    return {"layers": layers, "nodes": nodes,
            "inputs": [[model._nodes.index(v.node), v.index] for v in model.inputs],
            "outputs": [[model._nodes.index(v.node), v.index] for v in model.outputs],
            "multi_out": model._multi_out}


def build_layer(cfg):
    from zoo.pipeline.api.keras.engine.topology import Model, Sequential
    cls = _resolve(*cfg["class"])
    if "sequential" in cfg:
        m = cls(name=cfg.get("name"))
        for i, c in enumerate(cfg["sequential"]):
            l = build_layer(c)
            if i == 0 and l._given_input_shape is None and cfg.get("input_shape") is not None:
                l._given_input_shape = tuple(cfg["input_shape"])
            m.add(l)
        return m
    if "graph" in cfg:
        return build_graph(cfg["graph"], cls, cfg.get("name"))
    layer = cls(*[_dec(x) for x in cfg["args"]], **{k: _dec(v) for k, v in cfg["kwargs"].items()})
    gis = cfg.get("given_input_shape")
    if gis is not None and layer._given_input_shape is None:
        g = _dec(gis)
        layer._given_input_shape = tuple(g) if g and not isinstance(g[0], (list, tuple)) else g
    bs = cfg.get("built_shape")
    if bs is not None and not layer.built:
        shape = _dec(bs)
        layer._ensure_built(tuple(shape))
    return layer


def build_graph(g, cls=None, name=None):
    from zoo.pipeline.api.keras.engine.topology import Model
    layers = [build_layer(c) for c in g["layers"]]
    vals = []
    for n in g["nodes"]:
        if n.get("input"):
            vals.append([Input(shape=tuple(n["shape"]), name=n["name"])])
            continue
        args = [vals[i][j] for i, j in n["inbound"]]
        out = layers[n["layer"]](args if (len(args) > 1 or n["list_input"]) else args[0])
        vals.append(out if isinstance(out, list) else [out])
    ins = [vals[i][j] for i, j in g["inputs"]]
    outs = [vals[i][j] for i, j in g["outputs"]]
    cls = cls or Model
    return cls(ins if len(ins) > 1 else ins[0], outs if g["multi_out"] else outs[0], name=name)


def save_model(model, path, over_write=False, format="bigdl"):
    """``format="bigdl"`` (default): the reference's BigDL/Zoo ``.model`` protobuf
    (zoo.utils.bigdl_model); ``"zoo"``: the framework's torch-file config format."""
    import os
    if os.path.exists(path) and not over_write:
        raise FileExistsError("%s exists; pass over_write=True" % path)
    if format == "bigdl":
        from zoo.utils.bigdl_model import save_bigdl_model
        save_bigdl_model(model, path, over_write=True)
        return
    from zoo.utils.checkpoint import save_object
    state = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    save_object({"format": FORMAT, "arch": layer_config(model), "state": state}, path, True)


def load_model(path):
    """Reads both the BigDL/Zoo ``.model`` protobuf and the torch-file format."""
    from zoo.utils.bigdl_model import is_bigdl_model_file, load_bigdl_model
    if is_bigdl_model_file(path):
        return load_bigdl_model(path)
    from zoo.utils.checkpoint import load_object
    d = load_object(path)
    if not isinstance(d, dict) or d.get("format") != FORMAT:
        raise ValueError("%s is not a zoo keras model file" % path)
    m = build_layer(d["arch"])
    m.load_state_dict(d["state"])
    return m
