"""Net loaders (NetSpec / test_net.py / test_inference_model.py analogues).

Fixtures are the reference's own files, read with the framework's protobuf
decoder (nothing in them is executed): models/bigdl/bigdl_lenet.model,
models/caffe/test_persist.{prototxt,caffemodel}, test.{prototxt,caffemodel}.
No reference outputs ship with them, so model outputs are checked against an
independent numpy/PyTorch recomputation from the decoded weights; end-to-end
numerical parity with BigDL itself is unpinned.
"""
import os
import threading

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from zoo.common.nncontext import init_nncontext

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "reference_models")  # vendored
PYREF = "/root/reference/pyzoo/test/zoo/resources"
need_ref = pytest.mark.skipif(not os.path.exists(REF), reason="reference fixtures not present")


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


@need_ref
def test_load_bigdl_lenet_graph_ops():
    from zoo.pipeline.api.keras.models import Sequential
    from zoo.pipeline.api.net import Net
    model = Net.load_bigdl(os.path.join(REF, "bigdl/bigdl_lenet.model"))
    assert len(model.layers) == 12
    assert len(Sequential().add(model).flattened_layers()) == 12
    sub = model.new_graph(["reshape2"])
    sub.freeze_up_to(["pool3"])
    assert not any(p.requires_grad for p in sub.node("conv1_5x5").parameters())
    sub.unfreeze()
    assert all(p.requires_grad for p in sub.parameters())
    assert sub.forward_numpy(np.zeros([1, 1, 28, 28])).shape == (1, 192)
    x = np.random.rand(4, 28, 28, 1).astype(np.float32)
    out = model.forward_numpy(x)
    assert out.shape == (4, 5)
    assert np.allclose(np.exp(out).sum(1), 1.0, atol=1e-5)  # LogSoftMax head
    # independent recomputation from the decoded weights
    n = {k: model.node(k).op for k in model.node_names}
    t = torch.from_numpy(x).reshape(4, 1, 28, 28)
    # graph edges of the fixture: conv1 -> tanh1 -> pool1 -> tanh2 -> conv2 -> pool3 -> reshape2 -> fc1 ...
    h = torch.tanh(F.max_pool2d(torch.tanh(F.conv2d(t, n["conv1_5x5"].weight, n["conv1_5x5"].bias)), 2))
    h = F.max_pool2d(F.conv2d(h, n["conv2_5x5"].weight, n["conv2_5x5"].bias), 2)
    h = torch.tanh(F.linear(h.reshape(4, 192), n["fc1"].weight, n["fc1"].bias))
    ref = F.log_softmax(F.linear(h, n["fc2"].weight, n["fc2"].bias), -1)
    assert np.allclose(out, ref.detach().numpy(), atol=1e-5)
    assert float(n["conv1_5x5"].weight.abs().sum()) > 0


def _caffe_blobs(path):
    from zoo.pipeline.api.net.caffe_loader import read_caffemodel
    return read_caffemodel(path)


@need_ref
def test_load_caffe_matches_numpy_recompute():
    from zoo.pipeline.api.net import Net
    d, w = os.path.join(PYREF, "test.prototxt"), os.path.join(PYREF, "test.caffemodel")
    model = Net.load_caffe(d, w)
    b = _caffe_blobs(w)
    x = np.random.rand(2, 3, 5, 5).astype(np.float32)
    t = torch.from_numpy(x)
    h = F.conv2d(t, torch.from_numpy(b["conv"][0]), torch.from_numpy(b["conv"][1].reshape(-1)))
    h = F.conv2d(h, torch.from_numpy(b["conv2"][0]), torch.from_numpy(b["conv2"][1].reshape(-1))
                 if len(b["conv2"]) > 1 else None)
    ref = h.reshape(2, -1) @ torch.from_numpy(b["ip"][0].reshape(2, -1)).t()
    assert np.allclose(model.forward_numpy(x), ref.numpy(), atol=1e-5)
    pm = Net.load_caffe(os.path.join(REF, "caffe/test_persist.prototxt"),
                        os.path.join(REF, "caffe/test_persist.caffemodel"))
    sub = pm.new_graph(["ip"])
    sub.freeze_up_to(["conv2"])
    sub.unfreeze()
    out = pm.forward_numpy(np.random.rand(2, 3, 5, 5).astype(np.float32))
    assert out.shape == (2, 2) and np.allclose(out.sum(1), 1.0, atol=1e-5)  # Softmax head


def test_bigdl_encode_decode_roundtrip(tmp_path):
    from zoo.pipeline.api.net import Net
    from zoo.utils.bigdl_proto import encode_module
    rng = np.random.default_rng(0)
    w1, b1 = rng.standard_normal((8, 6)).astype(np.float32), rng.standard_normal(8).astype(np.float32)
    w2, b2 = rng.standard_normal((3, 8)).astype(np.float32), rng.standard_normal(3).astype(np.float32)
    spec = {"name": "seq", "type": "com.intel.analytics.bigdl.nn.Sequential", "submodules": [
        {"name": "l1", "type": "com.intel.analytics.bigdl.nn.Linear", "weight": w1, "bias": b1,
         "attr": {"inputSize": 6, "outputSize": 8, "withBias": True}},
        {"name": "r", "type": "com.intel.analytics.bigdl.nn.ReLU", "attr": {}},
        {"name": "l2", "type": "com.intel.analytics.bigdl.nn.Linear", "weight": w2, "bias": b2,
         "attr": {"inputSize": 8, "outputSize": 3, "withBias": True}}]}
    p = tmp_path / "m.model"
    p.write_bytes(encode_module(spec))
    m = Net.load_bigdl(str(p))
    x = rng.standard_normal((5, 6)).astype(np.float32)
    ref = np.maximum(x @ w1.T + b1, 0) @ w2.T + b2
    assert np.allclose(m.forward_numpy(x), ref, atol=1e-5)


def test_onnx_loader_against_torch(tmp_path):
    from zoo.pipeline.api.net import Net
    from zoo.pipeline.api.onnx.onnx_loader import enc_node, make_model
    rng = np.random.default_rng(1)
    wc = rng.standard_normal((4, 3, 3, 3)).astype(np.float32) * 0.3
    bc = rng.standard_normal(4).astype(np.float32)
    wg = rng.standard_normal((5, 4 * 4 * 4)).astype(np.float32) * 0.1
    bg = rng.standard_normal(5).astype(np.float32)
    scale, bias = np.ones(4, np.float32) * 1.5, np.full(4, 0.1, np.float32)
    mean, var = np.full(4, 0.2, np.float32), np.full(4, 2.0, np.float32)
    nodes = [enc_node("Conv", ["x", "wc", "bc"], ["c"], "conv", kernel_shape=[3, 3], pads=[1, 1, 1, 1]),
             enc_node("BatchNormalization", ["c", "s", "b", "m", "v"], ["bn"], "bn", epsilon=1e-5),
             enc_node("Relu", ["bn"], ["r"], "relu"),
             enc_node("MaxPool", ["r"], ["p"], "pool", kernel_shape=[2, 2], strides=[2, 2]),
             enc_node("Flatten", ["p"], ["f"], "flat", axis=1),
             enc_node("Gemm", ["f", "wg", "bg"], ["g"], "fc", transB=1),
             enc_node("Softmax", ["g"], ["y"], "sm", axis=1)]
    data = make_model(nodes, [("x", [1, 3, 8, 8])], [("y", [1, 5])],
                      {"wc": wc, "bc": bc, "wg": wg, "bg": bg, "s": scale, "b": bias, "m": mean, "v": var})
    p = tmp_path / "m.onnx"
    p.write_bytes(data)
    g = Net.load_onnx(str(p))
    x = rng.standard_normal((2, 3, 8, 8)).astype(np.float32)
    t = torch.from_numpy(x)
    h = F.conv2d(t, torch.from_numpy(wc), torch.from_numpy(bc), padding=1)
    h = (h - 0.2) / np.sqrt(2.0 + 1e-5) * 1.5 + 0.1
    h = F.max_pool2d(torch.relu(h), 2).reshape(2, -1)
    ref = torch.softmax(h @ torch.from_numpy(wg).t() + torch.from_numpy(bg), 1)
    assert np.allclose(g.forward_numpy(x), ref.numpy(), atol=1e-5)


def test_torchnet_trains_through_keras_api():
    from zoo.pipeline.api.net import TorchCriterion, TorchNet
    torch.manual_seed(0)
    mod = torch.nn.Sequential(torch.nn.Linear(4, 16), torch.nn.Tanh(), torch.nn.Linear(16, 1))
    net = TorchNet.from_pytorch(mod, input_shape=(4,))
    x = np.random.rand(128, 4).astype(np.float32)
    y = (x.sum(1, keepdims=True) * 0.5).astype(np.float32)
    net.compile(optimizer="adam", loss=TorchCriterion.from_pytorch(torch.nn.MSELoss()))
    before = net.evaluate(x, y)[0]
    net.fit(x, y, batch_size=16, nb_epoch=20)
    assert net.evaluate(x, y)[0] < 0.2 * before


@need_ref
def test_inference_model_bigdl_caffe_threads():
    from zoo.pipeline.api.net import Net
    from zoo.pipeline.inference import InferenceModel
    im = InferenceModel(3)
    im.load_bigdl(os.path.join(REF, "bigdl/bigdl_lenet.model"))
    x = np.random.rand(4, 28, 28, 1).astype(np.float32)
    ref = Net.load_bigdl(os.path.join(REF, "bigdl/bigdl_lenet.model")).forward_numpy(x)
    results = [None] * 6

    def worker(i):
        results[i] = im.predict(x)
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for r in results:
        assert np.allclose(r, ref, atol=1e-5)
    ic = InferenceModel(2, auto_scaling=True)
    ic.load_caffe(os.path.join(REF, "caffe/test_persist.prototxt"), os.path.join(REF, "caffe/test_persist.caffemodel"))
    assert ic.predict(np.random.rand(4, 3, 8, 8)).shape[1] == 2


def test_inference_model_module_and_batches():
    from zoo.pipeline.inference import InferenceModel
    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.ReLU())
    im = InferenceModel(2, max_batch=5).load_module(m)
    x = np.random.rand(12, 3).astype(np.float32)
    with torch.no_grad():
        ref = m(torch.from_numpy(x)).numpy()
    assert np.allclose(im.predict(x), ref, atol=1e-6)
    assert (im.predict_classes(x) == ref.argmax(1)).all()
