"""Keras 1.2 / 2.x model import and Keras 2 export (N1 ``Net.load_keras``, K1
``saveToKeras2``).

The reference builds the model through BigDL's Keras converter (DefinitionLoader /
WeightLoader over keras + h5py; Py/pipeline/api/net/net_load.py:127-138) and exports
with ``KerasNet.saveToKeras2`` (Topology.scala). Here the JSON definition is mapped
onto this framework's Keras layers directly and the HDF5 weight files are read and
written with the built-in HDF5 codec (``zoo.util.hdf5``; no h5py).

Supported layers: InputLayer, Dense, Activation, Dropout, Flatten, Reshape, Permute,
RepeatVector, Conv2D/Convolution2D, MaxPooling2D/AveragePooling2D (+1D), Global
Average/Max Pooling 1D/2D, ZeroPadding2D, BatchNormalization, Embedding, SimpleRNN,
LSTM, GRU, and the merges (Merge, Add, Multiply, Average, Maximum, Concatenate) in
Sequential and functional (Model) graphs. Weight layouts: Dense kernels (in, out),
Conv2D kernels (rows, cols, in, out) for channels_last / (out, in, rows, cols) for
Keras-1 "th", LSTM/GRU concatenated (Keras 2 / Keras 1 consume_less="gpu") or per-gate
(Keras 1, order i, c, f, o) arrays.
"""
import json

import numpy as np
import torch

from zoo.pipeline.api.keras import layers as L
from zoo.pipeline.api.keras.engine.topology import Merge, Model, Sequential

_ACT = {"linear": None, None: None}


def _act(name):
    return _ACT.get(name, name)


def _shape(cfg):
    s = cfg.get("batch_input_shape")
    if s is not None:
        return tuple(s[1:])
    if cfg.get("input_dim") is not None:
        return (cfg["input_dim"],)
    return None


def _ordering(cfg):
    df = cfg.get("data_format") or cfg.get("dim_ordering")
    return "th" if df in ("channels_first", "th") else "tf"


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)


class _Conv:
    """(layer, weight setter) for one Keras layer config."""

    @staticmethod
    def build(cls, cfg):  # noqa: C901 - one table
        kw = {"name": cfg.get("name")}
        shp = _shape(cfg)
        if shp is not None:
            kw["input_shape"] = shp
        if cls == "InputLayer":
            return None, None
        if cls == "Dense":
            units = cfg.get("units", cfg.get("output_dim"))
            lay = L.Dense(units, activation=_act(cfg.get("activation")), bias=cfg.get("use_bias", cfg.get("bias", True)),
                          **kw)

            def setw(ws):
                with torch.no_grad():
                    lay.weight.copy_(torch.as_tensor(np.asarray(ws[0]).T.copy()))
                    if lay.bias is not None and len(ws) > 1:
                        lay.bias.copy_(torch.as_tensor(np.asarray(ws[1])))
            return lay, setw
        if cls == "Activation":
            return L.Activation(cfg["activation"], **kw), None
        if cls == "Dropout":
            return L.Dropout(cfg.get("rate", cfg.get("p", 0.5)), **kw), None
        if cls == "Flatten":
            return L.Flatten(**kw), None
        if cls == "Reshape":
            return L.Reshape(tuple(cfg["target_shape"]), **kw), None
        if cls == "Permute":
            return L.Permute(tuple(cfg["dims"]), **kw), None
        if cls == "RepeatVector":
            return L.RepeatVector(cfg["n"], **kw), None
        if cls in ("Conv2D", "Convolution2D"):
            if "filters" in cfg:
                f, (r, c) = cfg["filters"], _pair(cfg["kernel_size"])
                mode, sub = cfg.get("padding", "valid"), _pair(cfg.get("strides", 1))
            else:
                f, r, c = cfg["nb_filter"], cfg["nb_row"], cfg["nb_col"]
                mode, sub = cfg.get("border_mode", "valid"), _pair(cfg.get("subsample", 1))
            order = _ordering(cfg)
            lay = L.Convolution2D(f, r, c, activation=_act(cfg.get("activation")), border_mode=mode, subsample=sub,
                                  dim_ordering=order, bias=cfg.get("use_bias", cfg.get("bias", True)), **kw)

            def setw(ws):
                k = np.asarray(ws[0])
                if order == "th" and k.shape[0] != f and k.shape[-1] == f:   # Keras 2 kernel, channels_first
                    k = k.transpose(3, 2, 0, 1)
                lay.set_weights([k] + list(ws[1:]))
            return lay, setw
        if cls in ("MaxPooling2D", "AveragePooling2D"):
            pool = _pair(cfg.get("pool_size", 2))
            st = cfg.get("strides")
            mode = cfg.get("padding", cfg.get("border_mode", "valid"))
            klass = L.MaxPooling2D if cls.startswith("Max") else L.AveragePooling2D
            return klass(pool, _pair(st) if st is not None else None, mode, _ordering(cfg), **kw), None
        if cls in ("MaxPooling1D", "AveragePooling1D"):
            pl = cfg.get("pool_size", cfg.get("pool_length", 2))
            pl = pl[0] if isinstance(pl, (list, tuple)) else pl
            st = cfg.get("strides", cfg.get("stride"))
            st = st[0] if isinstance(st, (list, tuple)) else st
            klass = L.MaxPooling1D if cls.startswith("Max") else L.AveragePooling1D
            return klass(pl, st, cfg.get("padding", cfg.get("border_mode", "valid")), **kw), None
        if cls in ("GlobalAveragePooling2D", "GlobalMaxPooling2D"):
            return getattr(L, cls)(dim_ordering=_ordering(cfg), **kw), None
        if cls in ("GlobalAveragePooling1D", "GlobalMaxPooling1D"):
            return getattr(L, cls)(**kw), None
        if cls == "ZeroPadding2D":
            p = cfg.get("padding", (1, 1))
            p = tuple(x[0] if isinstance(x, (list, tuple)) else x for x in p)
            return L.ZeroPadding2D(p, dim_ordering=_ordering(cfg), **kw), None
        if cls == "BatchNormalization":
            axis = cfg.get("axis", -1)
            axis = axis[0] if isinstance(axis, (list, tuple)) else axis
            order = "th" if axis == 1 else "tf"
            lay = L.BatchNormalization(epsilon=cfg.get("epsilon", 1e-3), momentum=cfg.get("momentum", 0.99),
                                       dim_ordering=order, **kw)
            center, scale = cfg.get("center", True), cfg.get("scale", True)

            def setw(ws):
                ws = list(ws)
                gamma = ws.pop(0) if scale else None
                beta = ws.pop(0) if center else None
                mean, var = ws[0], ws[1]
                n = len(mean)
                lay.set_weights([gamma if gamma is not None else np.ones(n, np.float32),
                                 beta if beta is not None else np.zeros(n, np.float32), mean, var])
            return lay, setw
        if cls == "Embedding":
            lay = L.Embedding(cfg["input_dim"], cfg["output_dim"], input_length=cfg.get("input_length"),
                              mask_zero=cfg.get("mask_zero", False), **kw)

            def setw(ws):
                with torch.no_grad():
                    lay.embeddings.copy_(torch.as_tensor(np.asarray(ws[0])))
            return lay, setw
        if cls in ("LSTM", "GRU", "SimpleRNN"):
            units = cfg.get("units", cfg.get("output_dim"))
            args = dict(activation=cfg.get("activation", "tanh"), return_sequences=cfg.get("return_sequences", False),
                        go_backwards=cfg.get("go_backwards", False), **kw)
            if cls != "SimpleRNN":
                args["inner_activation"] = cfg.get("recurrent_activation", cfg.get("inner_activation",
                                                                                   "hard_sigmoid"))
            lay = getattr(L, cls)(units, **args)
            gates = {"LSTM": 4, "GRU": 3, "SimpleRNN": 1}[cls]

            def setw(ws):
                ws = [np.asarray(w) for w in ws]
                if len(ws) == 3 * gates and gates > 1:      # Keras 1 per-gate: (W, U, b) per gate
                    order = ["i", "c", "f", "o"] if cls == "LSTM" else ["z", "r", "h"]
                    want = ["i", "f", "c", "o"] if cls == "LSTM" else ["z", "r", "h"]
                    per = {g: ws[3 * k:3 * k + 3] for k, g in enumerate(order)}
                    W = np.concatenate([per[g][0] for g in want], 1)
                    U = np.concatenate([per[g][1] for g in want], 1)
                    b = np.concatenate([per[g][2] for g in want], 0)
                else:
                    W, U, b = ws[0], ws[1], (ws[2] if len(ws) > 2 else np.zeros(ws[0].shape[1], np.float32))
                with torch.no_grad():
                    lay.W.copy_(torch.as_tensor(W.T.copy()))
                    lay.U.copy_(torch.as_tensor(U.T.copy()))
                    lay.b.copy_(torch.as_tensor(b.reshape(-1)))
            return lay, setw
        merges = {"Add": "sum", "Multiply": "mul", "Average": "ave", "Maximum": "max", "Concatenate": "concat"}
        if cls in merges or cls == "Merge":
            mode = merges.get(cls) or cfg.get("mode", "sum")
            axis = cfg.get("axis", cfg.get("concat_axis", -1))
            return Merge(mode=mode, concat_axis=axis, name=cfg.get("name")), None
        raise NotImplementedError("Keras import: layer class %r is not supported" % cls)


def _layers_of(config):
    if isinstance(config, list):          # Keras 1 Sequential
        return config
    return config.get("layers", [])


def model_from_config(model_cfg):
    """Keras ``model.to_json()`` dict -> (zoo Keras model, {layer name: weight setter})."""
    cls = model_cfg["class_name"]
    cfg = model_cfg["config"]
    setters = {}
    if cls == "Sequential":
        m = Sequential(name=cfg.get("name") if isinstance(cfg, dict) else None)
        pending_shape = None
        for lc in _layers_of(cfg):
            c = dict(lc["config"])
            if lc["class_name"] == "InputLayer":
                pending_shape = tuple(c["batch_input_shape"][1:])
                continue
            if pending_shape is not None and "batch_input_shape" not in c:
                c["batch_input_shape"] = [None] + list(pending_shape)
                pending_shape = None
            lay, setw = _Conv.build(lc["class_name"], c)
            m.add(lay)
            if setw is not None:
                setters[c.get("name")] = setw
        return m, setters
    if cls in ("Model", "Functional"):
        nodes = {}
        for lc in cfg["layers"]:
            c = dict(lc["config"])
            name = lc.get("name", c.get("name"))
            if lc["class_name"] == "InputLayer":
                nodes[name] = L.Input(shape=tuple(c["batch_input_shape"][1:]), name=name)
                continue
            c.pop("batch_input_shape", None)
            lay, setw = _Conv.build(lc["class_name"], c)
            inbound = lc.get("inbound_nodes") or []
            srcs = [nodes[e[0]] for e in inbound[0]] if inbound else []
            nodes[name] = lay(srcs if len(srcs) > 1 or isinstance(lay, Merge) else srcs[0])
            if setw is not None:
                setters[name] = setw
        ins = [nodes[x[0]] for x in cfg["input_layers"]]
        outs = [nodes[x[0]] for x in cfg["output_layers"]]
        return Model(ins if len(ins) > 1 else ins[0], outs if len(outs) > 1 else outs[0]), setters
    raise NotImplementedError("Keras import: model class %r" % cls)


def _as_str(v):
    if isinstance(v, (bytes, np.bytes_)):
        return bytes(v).decode("utf-8")
    return str(v)


def load_weights_hdf5(setters, h5, by_name=False):
    """Keras weight file layout: root (or ``model_weights``) attrs ``layer_names``; each
    layer group holds ``weight_names`` datasets."""
    g = h5["model_weights"] if "model_weights" in h5 else h5
    names = [_as_str(n) for n in np.atleast_1d(g.attrs.get("layer_names", np.array([])))]
    if not names:
        names = list(g.keys())
    loaded = 0
    for n in names:
        if n not in g:
            continue
        lg = g[n]
        wnames = [_as_str(w) for w in np.atleast_1d(lg.attrs.get("weight_names", np.array([])))]
        if not wnames:
            continue
        if n not in setters:
            if by_name:
                continue
            raise ValueError("Keras import: weights for layer %r but no such layer in the model" % n)
        setters[n]([np.asarray(lg[w].read()) for w in wnames])
        loaded += 1
    return loaded


def load_keras(json_path=None, hdf5_path=None, by_name=False):
    """Net.load_keras: definition from ``json_path`` (or the ``model_config`` of a full-model
    HDF5 file) and weights from ``hdf5_path``."""
    from zoo.util.hdf5 import File
    h5 = File(hdf5_path) if hdf5_path else None
    if json_path:
        with open(json_path) as f:
            model_cfg = json.load(f)
    elif h5 is not None and "model_config" in h5.attrs:
        model_cfg = json.loads(_as_str(h5.attrs["model_config"]))
    else:
        raise ValueError("load_keras needs a json definition or a full-model HDF5 file")
    model, setters = model_from_config(model_cfg)
    if h5 is not None:
        load_weights_hdf5(setters, h5, by_name)
    return model


# ---------------------------------------------------------------------------
# export (saveToKeras2)
# ---------------------------------------------------------------------------
def _export_layer(lay, first_shape=None):  # noqa: C901
    c = {"name": lay.name, "trainable": True}
    if first_shape is not None:
        c["batch_input_shape"] = [None] + list(first_shape)
    act = getattr(lay, "activation", None)
    act = act if isinstance(act, str) else ("linear" if act is None else getattr(act, "__name__", "linear"))
    if isinstance(lay, L.Dense):
        c.update(units=lay.output_dim, activation=act, use_bias=lay.bias is not None)
        ws = [lay.weight.detach().float().cpu().numpy().T.copy()]
        if lay.bias is not None:
            ws.append(lay.bias.detach().float().cpu().numpy().copy())
        return "Dense", c, ws, ["kernel:0", "bias:0"][:len(ws)]
    if isinstance(lay, L.Convolution2D):
        order = "channels_first" if lay.dim_ordering == "th" else "channels_last"
        c.update(filters=lay.nb_filter, kernel_size=list(lay.kernel), strides=list(lay.subsample),
                 padding=lay.border_mode if isinstance(lay.border_mode, str) else "valid", data_format=order,
                 activation=act, use_bias=lay.bias is not None, dilation_rate=list(lay.dilation))
        ws = lay.get_weights()
        if lay.dim_ordering == "th":   # Keras 2 kernels are (rows, cols, in, out) in both formats
            ws[0] = ws[0].transpose(2, 3, 1, 0)
        return "Conv2D", c, ws, ["kernel:0", "bias:0"][:len(ws)]
    if isinstance(lay, (L.MaxPooling2D, L.AveragePooling2D)):
        c.update(pool_size=list(lay.pool_size), strides=list(lay.strides), padding=lay.border_mode,
                 data_format="channels_first" if lay.dim_ordering == "th" else "channels_last")
        return ("MaxPooling2D" if isinstance(lay, L.MaxPooling2D) else "AveragePooling2D"), c, [], []
    if isinstance(lay, L.BatchNormalization):
        c.update(axis=1 if lay.dim_ordering == "th" else -1, epsilon=lay.epsilon, momentum=lay.momentum,
                 center=True, scale=True)
        return "BatchNormalization", c, lay.get_weights(), ["gamma:0", "beta:0", "moving_mean:0",
                                                           "moving_variance:0"]
    if isinstance(lay, L.Dropout):
        c.update(rate=lay.p)
        return "Dropout", c, [], []
    if isinstance(lay, L.Flatten):
        return "Flatten", c, [], []
    if isinstance(lay, L.Activation):
        c.update(activation=act)
        return "Activation", c, [], []
    if isinstance(lay, L.Reshape):
        c.update(target_shape=list(lay.target_shape))
        return "Reshape", c, [], []
    if isinstance(lay, L.Embedding):
        c.update(input_dim=lay.input_dim, output_dim=lay.output_dim)
        return "Embedding", c, [lay.embeddings.detach().float().cpu().numpy().copy()], ["embeddings:0"]
    for cls in ("LSTM", "GRU", "SimpleRNN"):
        if type(lay).__name__ == cls:
            c.update(units=lay.output_dim, activation=lay.activation, return_sequences=lay.return_sequences,
                     go_backwards=lay.go_backwards)
            if cls != "SimpleRNN":
                c["recurrent_activation"] = lay.inner_activation
            ws = [lay.W.detach().float().cpu().numpy().T.copy(), lay.U.detach().float().cpu().numpy().T.copy(),
                  lay.b.detach().float().cpu().numpy().copy()]
            return cls, c, ws, ["kernel:0", "recurrent_kernel:0", "bias:0"]
    if type(lay).__name__ in ("GlobalAveragePooling2D", "GlobalMaxPooling2D"):
        c.update(data_format="channels_first" if lay.dim_ordering == "th" else "channels_last")
        return type(lay).__name__, c, [], []
    raise NotImplementedError("saveToKeras2: layer %s (%s) has no Keras 2 counterpart here"
                              % (lay.name, type(lay).__name__))


def save_keras2(model, json_path=None, hdf5_path=None):
    """Write a Sequential model as a Keras 2 definition (json) and/or a Keras 2 full-model
    HDF5 file (``model_config`` attribute + ``model_weights`` groups)."""
    from zoo.util.hdf5 import Writer
    if not isinstance(model, Sequential):
        raise NotImplementedError("saveToKeras2 supports Sequential models")
    layers_cfg, weights = [], []
    first = tuple(model.get_input_shape()[1:])
    for i, lay in enumerate(model.stack):
        cls, cfg, ws, wn = _export_layer(lay, first if i == 0 else None)
        layers_cfg.append({"class_name": cls, "config": cfg})
        weights.append((lay.name, ws, wn))
    model_cfg = {"class_name": "Sequential", "config": {"name": model.name, "layers": layers_cfg},
                 "keras_version": "2.2.4", "backend": "tensorflow"}
    if json_path:
        with open(json_path, "w") as f:
            json.dump(model_cfg, f)
    if hdf5_path:
        w = Writer()
        w.attrs()["model_config"] = json.dumps(model_cfg)
        w.attrs()["keras_version"] = "2.2.4"
        w.attrs()["backend"] = "tensorflow"
        w.create_group("model_weights")
        w.attrs("model_weights")["layer_names"] = np.array([n.encode() for n, _, _ in weights])
        for name, ws, wn in weights:
            w.create_group("model_weights/" + name)
            w.attrs("model_weights/" + name)["weight_names"] = np.array(
                [("%s/%s" % (name, x)).encode() for x in wn] if wn else [], dtype="S1" if not wn else None)
            for arr, x in zip(ws, wn):
                w.create_dataset("model_weights/%s/%s/%s" % (name, name, x), np.asarray(arr, np.float32))
        w.save(hdf5_path)
    return model_cfg
