"""TFNet: TF GraphDef / SavedModel executed on torch (reference tests:
zoo/src/test/scala/.../pipeline/api/net/TFNetSpec.scala, pyzoo/test/zoo/tfpark/test_tfnet.py).

Fixtures are the reference's own serialized graphs, decoded with the safe
protobuf codec (nothing in them is executed as code). TensorFlow itself is not
installed, so outputs are pinned against (a) the graph's constants evaluated by
hand in numpy and (b) TF's own exported gradient sub-graph (tfnet_training).
"""
import os

import numpy as np
import pytest
import torch

from zoo.tfpark import TFNet
from zoo.pipeline.api.net.tf_graph import parse_graph_def, read_sstable, read_tensor_bundle

R = "/root/reference/zoo/src/test/resources"
PYR = "/root/reference/pyzoo/test/zoo/resources"
pytestmark = pytest.mark.skipif(not os.path.isdir(R), reason="reference fixtures not mounted")


def _consts(path):
    nodes = parse_graph_def(open(path, "rb").read())
    return {n.name: n.attr["value"] for n in nodes if n.op == "Const"}


def test_export_folder_forward_matches_numpy():
    net = TFNet.from_export_folder(os.path.join(PYR, "tfnet"))
    x = np.random.rand(2, 4).astype(np.float32)
    out = net.forward_numpy(x)
    assert out.shape == (2, 2)
    c = _consts(os.path.join(PYR, "tfnet", "frozen_inference_graph.pb"))
    h = np.maximum(x @ c["dense/kernel"] + c["dense/bias"], 0)
    ref = 1 / (1 + np.exp(-(h @ c["dense_1/kernel"] + c["dense_1/bias"])))
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


def test_shrunk_input_and_clone():
    import copy
    net = TFNet(os.path.join(R, "tfnet"))
    x = np.random.rand(4, 4).astype(np.float32)[:2]
    out = net.forward_numpy(x)
    assert out.shape == (2, 2)
    np.testing.assert_array_equal(copy.deepcopy(net).forward_numpy(x), out)


def test_multi_type_inputs_outputs_and_input_check():
    ins = ["float_input:0", "double_input:0", "int_input:0", "long_input:0", "uint8_input:0"]
    outs = ["float_output:0", "double_output:0", "int_output:0", "long_output:0", "uint8_output:0"]
    net = TFNet(os.path.join(R, "tf", "multi_type_inputs_outputs.pb"), ins, outs)
    data = [np.array([[1.0]]), np.array([[2.0]]), np.array([[3.0]]), np.array([[4.0]]), np.array([[255.0]])]
    res = net.forward_numpy(data)
    assert [r.dtype for r in res] == [np.float32, np.float64, np.int32, np.int64, np.uint8]
    for r, d in zip(res, data):
        assert float(r.reshape(-1)[0]) == float(d.reshape(-1)[0])
    grads = net.backward(data, [None] * 5)
    assert all(float(np.sum(g)) == 0.0 for g in grads)
    with pytest.raises(ValueError):
        net.forward_numpy(data[:4])
    with pytest.raises(ValueError):
        net.forward_numpy(data[:1])


def test_backward_matches_tf_exported_gradient_graph():
    """TFNetSpec 'work with backward': our autograd gradient equals what TF's own
    exported gradient ops (SigmoidGrad/ReluGrad/BiasAddGrad/MatMul) compute."""
    folder = os.path.join(R, "tfnet_training")
    net = TFNet(folder)
    x = np.random.rand(2, 4).astype(np.float32)
    out = net.forward_numpy(x)
    gin = net.backward(x, out)
    assert gin.shape == x.shape
    meta = net.meta
    tf_grad = TFNet(os.path.join(folder, "frozen_inference_graph.pb"),
                    ["Placeholder:0", "dense_1/Sigmoid_grad:0"],
                    meta["grad_inputs"] + meta["grad_variables"])
    res = tf_grad.forward_numpy([x, out])
    np.testing.assert_allclose(gin, res[0], rtol=1e-5, atol=1e-6)
    assert [r.shape for r in res[1:]] == [(4, 10), (10,), (10, 2), (2,)]


def test_string_graph():
    net = TFNet(os.path.join(R, "tfnet_string"))
    out = net.forward_numpy(np.array([b"1.5", b"-3", b"42"], dtype=object))
    np.testing.assert_allclose(out, [1.5, -3.0, 42.0])


def test_saved_model_resource_variables():
    net = TFNet.from_saved_model(os.path.join(R, "saved-model-resource"), inputs=["flatten_input:0"],
                                 outputs=["dense_2/Softmax:0"])
    out = net.forward_numpy(np.ones((4, 28, 28, 1), np.float32))
    assert out.shape == (4, 10)
    np.testing.assert_allclose(out.sum(1), np.ones(4), rtol=1e-5)
    # weights came from the tensor bundle: recompute the MLP (dropout/BN are off at inference)
    v = read_tensor_bundle(os.path.join(R, "saved-model-resource", "variables", "variables"))
    assert v["dense/kernel"].shape == (784, 64)


def test_saved_model_signature_variants():
    p = os.path.join(R, "saved-model-signature")
    x = np.ones((4, 4), np.float32)
    a = TFNet.from_saved_model(p)
    assert a.input_names == ["Placeholder:0"] and a.forward_numpy(x).shape == (4, 10)
    b = TFNet.from_saved_model(p, inputs=["Placeholder:0"])
    c = TFNet.from_saved_model(p, outputs=["dense/BiasAdd:0"])
    np.testing.assert_allclose(b.forward_numpy(x), a.forward_numpy(x))
    np.testing.assert_allclose(c.forward_numpy(x), a.forward_numpy(x))
    v = read_tensor_bundle(os.path.join(p, "variables", "variables"))
    w, bias = v["dense/kernel"], v["dense/bias"]
    np.testing.assert_allclose(a.forward_numpy(x), x @ w + bias, rtol=1e-5, atol=1e-6)


def test_saved_model_missing_shard_uses_initializers():
    """saved-model-not-resource ships only variables.index (no data shard): the
    variables take their initializer values; the LeNet graph (Conv2D SAME,
    MaxPool, Reshape, MatMul) still runs end to end."""
    with pytest.warns(UserWarning):
        net = TFNet.from_saved_model(os.path.join(R, "saved-model-not-resource"), inputs=["Placeholder:0"],
                                     outputs=["LeNet/fc4/BiasAdd:0"])
    assert net.forward_numpy(np.ones((4, 28, 28, 1), np.float32)).shape == (4, 10)


def test_sstable_reader():
    entries = read_sstable(os.path.join(R, "saved-model-signature", "variables", "variables.index"))
    keys = [k for k, _ in entries]
    assert keys == sorted(keys) and b"dense/kernel" in keys


def test_conv_pool_ops_vs_reference_math():
    """Conv2D / MaxPool / AvgPool with TF SAME padding against explicit numpy."""
    from zoo.pipeline.api.net.tf_graph import Node, TFGraph
    x = torch.randn(1, 5, 5, 2)
    w = torch.randn(3, 3, 2, 4)
    nodes = [Node("x", "Placeholder", [], [], {"dtype": 1}), Node("w", "Const", [], [], {}),
             Node("c", "Conv2D", ["x", "w"], [], {"strides": [1, 2, 2, 1], "padding": b"SAME"}),
             Node("m", "MaxPool", ["x"], [], {"ksize": [1, 2, 2, 1], "strides": [1, 2, 2, 1], "padding": b"SAME"}),
             Node("a", "AvgPool", ["x"], [], {"ksize": [1, 2, 2, 1], "strides": [1, 2, 2, 1], "padding": b"SAME"})]
    g = TFGraph(nodes, {"w": w})
    c, m, a = g.run({"x": x}, ["c", "m", "a"])
    # SAME with stride 2 on 5: out 3, total pad 2 -> (1, 1)
    xp = torch.nn.functional.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1))
    ref = torch.nn.functional.conv2d(xp, w.permute(3, 2, 0, 1), stride=2).permute(0, 2, 3, 1)
    torch.testing.assert_close(c, ref)
    xn = x[0].numpy()
    # pool SAME on 5 with k2 s2: out 3, total pad 1 -> (0, 1): last window is the single edge row/col
    assert m.shape == (1, 3, 3, 2) and a.shape == (1, 3, 3, 2)
    np.testing.assert_allclose(m[0, 2, 2].numpy(), xn[4, 4])
    np.testing.assert_allclose(a[0, 0, 0].numpy(), xn[:2, :2].mean((0, 1)), rtol=1e-6)
    np.testing.assert_allclose(a[0, 2, 2].numpy(), xn[4, 4], rtol=1e-6)


def test_strided_slice_masks():
    from zoo.pipeline.api.net.tf_graph import Node, _strided_slice
    x = torch.arange(60).reshape(3, 4, 5)
    n = Node("s", "StridedSlice", [], [], {"begin_mask": 1, "end_mask": 0, "ellipsis_mask": 0,
                                           "new_axis_mask": 0, "shrink_axis_mask": 2})
    out = _strided_slice(n, x, [0, 1, 0], [2, 2, 5], [1, 1, 2])
    torch.testing.assert_close(out, x[:2, 1, 0:5:2])
    n2 = Node("s", "StridedSlice", [], [], {"begin_mask": 0, "end_mask": 0, "ellipsis_mask": 1,
                                            "new_axis_mask": 0, "shrink_axis_mask": 0})
    torch.testing.assert_close(_strided_slice(n2, x, [0, 1], [0, 3], [1, 1]), x[..., 1:3])
    n3 = Node("s", "StridedSlice", [], [], {"begin_mask": 1, "end_mask": 1, "ellipsis_mask": 0,
                                            "new_axis_mask": 0, "shrink_axis_mask": 0})
    torch.testing.assert_close(_strided_slice(n3, x, [0], [0], [-1]), x.flip(0))


def test_inference_model_load_tf():
    from zoo.pipeline.inference import InferenceModel
    m = InferenceModel(device="cpu").load_tf(os.path.join(PYR, "tfnet"))
    out = m.predict(np.random.rand(3, 4).astype(np.float32))
    assert np.asarray(out).shape == (3, 2)


@pytest.mark.gpu
def test_tfnet_on_gpu_matches_cpu(gpu):
    net = TFNet.from_saved_model(os.path.join(R, "saved-model-resource"), inputs=["flatten_input:0"],
                                 outputs=["dense_2/Softmax:0"])
    x = np.random.rand(8, 28, 28, 1).astype(np.float32)
    ref = net.forward_numpy(x)
    out = net.to(gpu).forward_numpy(x)
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5)


def test_export_tf_freezes_trained_variables(tmp_path):
    """zoo.util.tf.export_tf (Py/util/tf.py:50): a TFNet whose variables changed after
    loading is frozen (variables -> Const with the current values, resource reads ->
    Identity) into an export folder that loads back and computes the same outputs."""
    import torch
    from zoo.util.tf import export_tf
    p = os.path.join(R, "saved-model-signature")
    net = TFNet.from_saved_model(p, trainable=True)
    with torch.no_grad():
        for prm in net.parameters():
            prm.mul_(1.5).add_(0.25)        # "training" moved the weights
    x = np.random.rand(3, 4).astype(np.float32)
    want = net.forward_numpy(x)
    out = export_tf(net, str(tmp_path / "exp"), net.input_names, net.output_names)
    back = TFNet.from_export_folder(out)
    assert not list(back.parameters())      # nothing left to train: everything is a Const
    np.testing.assert_allclose(back.forward_numpy(x), want, rtol=1e-6, atol=1e-6)
    # a frozen export folder re-exports to an equivalent folder
    net2 = TFNet.from_export_folder(os.path.join(PYR, "tfnet"))
    out2 = export_tf(net2, str(tmp_path / "exp2"), net2.input_names, net2.output_names)
    np.testing.assert_allclose(TFNet.from_export_folder(out2).forward_numpy(x[:, :4]), net2.forward_numpy(x[:, :4]),
                               rtol=1e-6)
    with pytest.raises(TypeError):
        export_tf(object(), str(tmp_path / "bad"), [], [])


def test_tf_conv2d_native_path_geometry_on_cpu_reference():
    """The SAME / VALID / strided Conv2D geometry the native path reproduces (CPU check of
    the padding arithmetic it shares with the reference path)."""
    import torch
    from zoo.pipeline.api.net.tf_graph import Node, _conv2d
    x = torch.randn(2, 9, 9, 3)
    w = torch.randn(3, 3, 3, 5)
    for pad, st in (("SAME", 1), ("SAME", 2), ("VALID", 2)):
        n = Node("c", "Conv2D", [], [], {"strides": [1, st, st, 1], "padding": pad, "data_format": "NHWC"})
        y = _conv2d(n, x, w)
        exp = (9 + st - 1) // st if pad == "SAME" else (9 - 3) // st + 1
        assert y.shape == (2, exp, exp, 5)

