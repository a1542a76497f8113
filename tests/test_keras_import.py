"""N1 Net.load_keras / K1 saveToKeras2: Keras definitions (Keras 1.2 and 2.x json) and
HDF5 weight files through the built-in HDF5 codec (zoo/util/hdf5.py). The reader is also
checked on HDF5 files written by the HDF5 library itself when the image carries any
(PyTables' test data); parity of imported weights is pinned by recomputation in numpy."""
import glob
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def test_hdf5_writer_reader_roundtrip(tmp_path):
    from zoo.util import hdf5
    w = hdf5.Writer()
    a = np.random.RandomState(0).randn(3, 4).astype(np.float32)
    w.create_dataset("g/sub/x", a)
    w.create_dataset("g/i", np.arange(5, dtype=np.int64))
    for i in range(40):                       # more entries than one default symbol-table node
        w.create_dataset("many/d%02d" % i, np.full((2,), i, np.float64))
    w.attrs()["s"] = "hello"
    w.attrs("g")["names"] = np.array([b"a", b"bcd"])
    w.attrs("g/sub")["scalar"] = np.float32(2.5)
    w.save(str(tmp_path / "t.h5"))
    f = hdf5.File(str(tmp_path / "t.h5"))
    assert sorted(f.keys()) == ["g", "many"]
    assert np.array_equal(f["g/sub/x"].read(), a) and f["g/i"].read().tolist() == [0, 1, 2, 3, 4]
    assert len(f["many"].keys()) == 40 and f["many/d39"].read().tolist() == [39.0, 39.0]
    assert f.attrs["s"] == b"hello" and list(f["g"].attrs["names"]) == [b"a", b"bcd"]
    assert float(f["g/sub"].attrs["scalar"]) == 2.5


_LIB_FILES = sorted(glob.glob("/opt/conda/lib/python3.*/site-packages/tables/tests/smpl_*.h5"))


@pytest.mark.skipif(not _LIB_FILES, reason="no library-written HDF5 sample files in this image")
def test_hdf5_reader_on_library_written_files():
    from zoo.util import hdf5
    seen = 0
    for fn in _LIB_FILES:
        base = os.path.basename(fn)
        if not any(t in base for t in ("f64", "i32", "i64", "SDSextendible")):
            continue
        a = hdf5.File(fn)[hdf5.File(fn).keys()[0]].read()
        if "extendible" in base:
            assert a.shape == (10, 5)
        else:
            # PyTables smpl_* arrays: rows i hold i..i+4
            assert a.shape == (6, 5) and np.array_equal(a, np.arange(6)[:, None] + np.arange(5)[None, :])
        seen += 1
    assert seen >= 3


def _seq_model():
    from zoo.pipeline.api.keras.layers import (BatchNormalization, Convolution2D, Dense, Dropout, Flatten,
                                               MaxPooling2D)
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(0)
    m = Sequential()
    m.add(Convolution2D(4, 3, 3, activation="relu", border_mode="same", dim_ordering="tf", input_shape=(8, 8, 3)))
    m.add(BatchNormalization(dim_ordering="tf"))
    m.add(MaxPooling2D((2, 2), dim_ordering="tf"))
    m.add(Flatten())
    m.add(Dropout(0.3))
    m.add(Dense(5, activation="softmax"))
    return m


def test_save_to_keras2_and_load_keras_roundtrip(tmp_path):
    from zoo.pipeline.api.net import Net
    m = _seq_model()
    bn = m.stack[1]
    with torch.no_grad():
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 1.5)
    m.eval()
    x = torch.randn(2, 8, 8, 3)
    ref = m(x)
    js, h5 = str(tmp_path / "m.json"), str(tmp_path / "m.h5")
    cfg = m.save_to_keras2(json_path=js, hdf5_path=h5)
    assert [l["class_name"] for l in cfg["config"]["layers"]] == ["Conv2D", "BatchNormalization", "MaxPooling2D",
                                                                  "Flatten", "Dropout", "Dense"]
    m2 = Net.load_keras(hdf5_path=h5)           # full-model file: definition from model_config
    m2.eval()
    assert torch.allclose(m2(x), ref, atol=1e-5)
    m3 = Net.load_keras(json_path=js, hdf5_path=h5)
    m3.eval()
    assert torch.allclose(m3(x), ref, atol=1e-5)


def test_load_keras1_json_definition_and_per_gate_lstm(tmp_path):
    """A Keras 1.2 ``model.to_json()`` (Dense with output_dim / input_dim) and an LSTM whose
    weights come as Keras-1 per-gate arrays (order i, c, f, o)."""
    from zoo.pipeline.api.keras.keras_import import model_from_config
    from zoo.pipeline.api.keras.models import Sequential
    from zoo.pipeline.api.net import Net
    k1 = {"class_name": "Sequential", "config": [
        {"class_name": "Dense", "config": {"name": "dense_1", "output_dim": 32, "activation": "relu",
                                          "bias": True, "input_dim": 100, "batch_input_shape": [None, 100]}}]}
    p = tmp_path / "k1.json"
    p.write_text(json.dumps(k1))
    m = Net.load_keras(json_path=str(p))
    assert isinstance(m, Sequential) and m.get_output_shape() == (None, 32)
    # LSTM, Keras 1 per-gate weights
    r = np.random.RandomState(1)
    d, h = 3, 4
    per = {g: (r.randn(d, h).astype(np.float32), r.randn(h, h).astype(np.float32), r.randn(h).astype(np.float32))
           for g in "icfo"}
    cfg = {"class_name": "Sequential", "config": [
        {"class_name": "LSTM", "config": {"name": "lstm_1", "output_dim": h, "activation": "tanh",
                                         "inner_activation": "sigmoid", "return_sequences": False,
                                         "batch_input_shape": [None, 5, d]}}]}
    model, setters = model_from_config(cfg)
    setters["lstm_1"]([a for g in "icfo" for a in per[g]])
    x = r.randn(2, 5, d).astype(np.float32)
    sig = lambda v: 1 / (1 + np.exp(-v))  # noqa: E731
    hh, cc = np.zeros((2, h), np.float32), np.zeros((2, h), np.float32)
    for t in range(5):
        g = {k: x[:, t] @ per[k][0] + hh @ per[k][1] + per[k][2] for k in "icfo"}
        cc = sig(g["f"]) * cc + sig(g["i"]) * np.tanh(g["c"])
        hh = sig(g["o"]) * np.tanh(cc)
    model.eval()
    out = model(torch.from_numpy(x)).detach().numpy()
    assert np.allclose(out, hh, atol=1e-4)


def test_load_keras2_functional_model(tmp_path):
    from zoo.pipeline.api.keras.keras_import import model_from_config
    cfg = {"class_name": "Model", "config": {"name": "m", "layers": [
        {"name": "a", "class_name": "InputLayer", "config": {"name": "a", "batch_input_shape": [None, 6]},
         "inbound_nodes": []},
        {"name": "d1", "class_name": "Dense", "config": {"name": "d1", "units": 4, "activation": "tanh"},
         "inbound_nodes": [[["a", 0, 0, {}]]]},
        {"name": "d2", "class_name": "Dense", "config": {"name": "d2", "units": 4, "activation": "linear"},
         "inbound_nodes": [[["a", 0, 0, {}]]]},
        {"name": "cat", "class_name": "Concatenate", "config": {"name": "cat", "axis": -1},
         "inbound_nodes": [[["d1", 0, 0, {}], ["d2", 0, 0, {}]]]}],
        "input_layers": [["a", 0, 0]], "output_layers": [["cat", 0, 0]]}}
    model, setters = model_from_config(cfg)
    r = np.random.RandomState(2)
    k1, b1, k2, b2 = r.randn(6, 4), r.randn(4), r.randn(6, 4), r.randn(4)
    setters["d1"]([k1, b1])
    setters["d2"]([k2, b2])
    x = r.randn(3, 6).astype(np.float32)
    out = model(torch.from_numpy(x)).detach().numpy()
    ref = np.concatenate([np.tanh(x @ k1 + b1), x @ k2 + b2], 1)
    assert np.allclose(out, ref, atol=1e-5)


def test_torch7_t7_model_roundtrip(tmp_path):
    """Lua Torch7 binary serialisation (Net.loadTorch): an nn.Sequential LeNet-like model
    written in the .t7 format is decoded and rebuilt; outputs recomputed with torch ops."""
    from zoo.pipeline.api.net import Net
    from zoo.pipeline.api.net.torch7 import T7Object, load_torch7, read_t7, write_t7
    r = np.random.RandomState(5)
    cw = r.randn(6, 1 * 3 * 3).astype(np.float32) * 0.3    # SpatialConvolutionMM stores [out, in*kh*kw]
    cb = r.randn(6).astype(np.float32)
    lw = r.randn(10, 6 * 3 * 3).astype(np.float32) * 0.1
    lb = r.randn(10).astype(np.float32)
    bn = {"running_mean": r.randn(6).astype(np.float32), "running_var": (r.rand(6) + 0.5).astype(np.float32),
          "weight": r.randn(6).astype(np.float32), "bias": r.randn(6).astype(np.float32), "eps": 1e-5}
    mods = [T7Object("nn.SpatialConvolutionMM", {"nInputPlane": 1, "nOutputPlane": 6, "kW": 3, "kH": 3, "dW": 1,
                                                 "dH": 1, "padW": 1, "padH": 1, "weight": cw, "bias": cb}),
            T7Object("nn.SpatialBatchNormalization", bn),
            T7Object("nn.ReLU", {"inplace": False}),
            T7Object("nn.SpatialMaxPooling", {"kW": 2, "kH": 2, "dW": 2, "dH": 2, "padW": 0, "padH": 0}),
            T7Object("nn.View", {"size": np.array([54], np.int64)}),
            T7Object("nn.Linear", {"weight": lw, "bias": lb}),
            T7Object("nn.LogSoftMax", {})]
    model = T7Object("nn.Sequential", {"modules": mods, "train": False})
    p = str(tmp_path / "lenet.t7")
    write_t7(model, p)
    back = read_t7(p)
    assert back.cls == "nn.Sequential" and np.array_equal(back["modules"][1.0]["weight"], cw)
    m = load_torch7(p)
    x = torch.from_numpy(r.randn(2, 1, 6, 6).astype(np.float32))
    y = F.conv2d(x, torch.from_numpy(cw).reshape(6, 1, 3, 3), torch.from_numpy(cb), padding=1)
    y = F.batch_norm(y, torch.from_numpy(bn["running_mean"]), torch.from_numpy(bn["running_var"]),
                     torch.from_numpy(bn["weight"]), torch.from_numpy(bn["bias"]), False, 0.0, 1e-5)
    y = F.max_pool2d(F.relu(y), 2, 2).reshape(2, -1)
    ref = F.log_softmax(y @ torch.from_numpy(lw).t() + torch.from_numpy(lb), -1)
    with torch.no_grad():
        assert torch.allclose(m(x), ref, atol=1e-5)
    net = Net.load_torch(p)
    assert net is not None
