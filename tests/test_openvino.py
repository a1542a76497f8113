"""OpenVINO IR loader/executor (zoo/pipeline/inference/openvino.py) on hand-written IR
v10 and legacy v7 files (the reference's IR fixtures are downloaded at test time and
not in the tree, so parity is pinned against PyTorch recomputation of the same graph)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F


class _IR:
    """Tiny IR v10 writer for tests."""

    def __init__(self):
        self.layers, self.edges, self.blob = [], [], bytearray()
        self.nid = 0

    def _id(self):
        self.nid += 1
        return self.nid - 1

    def param(self, shape):
        i = self._id()
        dims = "".join("<dim>%d</dim>" % d for d in shape)
        self.layers.append('<layer id="%d" name="in%d" type="Parameter" version="opset1"><data shape="%s" '
                           'element_type="f32"/><output><port id="0" precision="FP32">%s</port></output></layer>'
                           % (i, i, ",".join(map(str, shape)), dims))
        return (i, 0)

    def const(self, arr):
        arr = np.ascontiguousarray(arr)
        et = {np.dtype(np.float32): "f32", np.dtype(np.int64): "i64", np.dtype(np.float16): "f16"}[arr.dtype]
        i = self._id()
        off = len(self.blob)
        self.blob += arr.tobytes()
        dims = "".join("<dim>%d</dim>" % d for d in arr.shape)
        self.layers.append('<layer id="%d" name="c%d" type="Const" version="opset1"><data element_type="%s" '
                           'shape="%s" offset="%d" size="%d"/><output><port id="0">%s</port></output></layer>'
                           % (i, i, et, ",".join(map(str, arr.shape)), off, arr.nbytes, dims))
        return (i, 0)

    def op(self, typ, inputs, attrs=None, nout=1):
        i = self._id()
        data = "" if not attrs else "<data %s/>" % " ".join('%s="%s"' % kv for kv in attrs.items())
        ins = "".join('<port id="%d"/>' % k for k in range(len(inputs)))
        outs = "".join('<port id="%d"/>' % (len(inputs) + k) for k in range(nout))
        self.layers.append('<layer id="%d" name="%s%d" type="%s" version="opset1">%s<input>%s</input>'
                           '<output>%s</output></layer>' % (i, typ.lower(), i, typ, data, ins, outs))
        for k, (fl, fp) in enumerate(inputs):
            self.edges.append('<edge from-layer="%d" from-port="%d" to-layer="%d" to-port="%d"/>' % (fl, fp, i, k))
        return (i, len(inputs))

    def result(self, x):
        i = self._id()
        self.layers.append('<layer id="%d" name="out%d" type="Result" version="opset1"><input><port id="0"/>'
                           '</input></layer>' % (i, i))
        self.edges.append('<edge from-layer="%d" from-port="%d" to-layer="%d" to-port="0"/>' % (x[0], x[1], i))

    def save(self, d):
        xml = '<?xml version="1.0"?><net name="t" version="10"><layers>%s</layers><edges>%s</edges></net>' % (
            "".join(self.layers), "".join(self.edges))
        with open(os.path.join(d, "m.xml"), "w") as f:
            f.write(xml)
        with open(os.path.join(d, "m.bin"), "wb") as f:
            f.write(bytes(self.blob))
        return os.path.join(d, "m.xml"), os.path.join(d, "m.bin")


def _cnn_ir(tmp_path, r):
    w1 = r.randn(8, 3, 3, 3).astype(np.float32) * 0.3
    b1 = r.randn(1, 8, 1, 1).astype(np.float32) * 0.1
    w2 = r.randn(16, 8, 3, 3).astype(np.float32) * 0.2
    fc = r.randn(5, 16 * 2 * 2).astype(np.float32) * 0.2
    fb = r.randn(1, 5).astype(np.float32) * 0.1
    ir = _IR()
    x = ir.param([2, 3, 8, 8])
    h = ir.op("Convolution", [x, ir.const(w1)], {"strides": "1,1", "dilations": "1,1", "pads_begin": "1,1",
                                                  "pads_end": "1,1", "auto_pad": "explicit"})
    h = ir.op("Add", [h, ir.const(b1)], {"auto_broadcast": "numpy"})
    h = ir.op("Relu", [h])
    h = ir.op("MaxPool", [h], {"strides": "2,2", "kernel": "2,2", "pads_begin": "0,0", "pads_end": "0,0",
                               "rounding_type": "floor"})
    h = ir.op("Convolution", [h, ir.const(w2)], {"strides": "2,2", "dilations": "1,1", "pads_begin": "0,0",
                                                  "pads_end": "0,0", "auto_pad": "same_upper"})
    h = ir.op("Clamp", [h], {"min": "0", "max": "6"})
    shp = ir.op("ShapeOf", [h])
    n = ir.op("Gather", [shp, ir.const(np.array([0], np.int64)), ir.const(np.array(0, np.int64))])
    tgt = ir.op("Concat", [n, ir.const(np.array([-1], np.int64))], {"axis": "0"})
    h = ir.op("Reshape", [h, tgt], {"special_zero": "false"})
    h = ir.op("MatMul", [h, ir.const(fc)], {"transpose_a": "false", "transpose_b": "true"})
    h = ir.op("Add", [h, ir.const(fb)], {"auto_broadcast": "numpy"})
    h = ir.op("SoftMax", [h], {"axis": "1"})
    ir.result(h)
    paths = ir.save(str(tmp_path))

    def ref(xt):
        y = F.relu(F.conv2d(xt, torch.from_numpy(w1), padding=1) + torch.from_numpy(b1))
        y = F.max_pool2d(y, 2, 2)
        y = F.pad(y, (0, 1, 0, 1))   # same_upper, k3 s2 on 4x4: total pad 1 -> (0, 1)
        y = torch.clamp(F.conv2d(y, torch.from_numpy(w2), stride=2), 0, 6)
        y = y.reshape(y.shape[0], -1) @ torch.from_numpy(fc).t() + torch.from_numpy(fb)
        return torch.softmax(y, 1)
    return paths, ref


def test_ir_v10_cnn_matches_torch(tmp_path):
    from zoo.pipeline.inference.openvino import load_openvino
    r = np.random.RandomState(0)
    (xml, binp), ref = _cnn_ir(tmp_path, r)
    m = load_openvino(xml, binp)
    x = torch.from_numpy(r.randn(2, 3, 8, 8).astype(np.float32))
    out = m.predict(x)
    assert out.shape == (2, 5)
    assert torch.allclose(out, ref(x), atol=1e-5)


def test_inference_model_load_openvino(tmp_path):
    from zoo.pipeline.inference import InferenceModel
    r = np.random.RandomState(1)
    (xml, binp), ref = _cnn_ir(tmp_path, r)
    im = InferenceModel()
    im.load_openvino(xml, binp)
    x = r.randn(2, 3, 8, 8).astype(np.float32)
    out = im.predict(x)
    out = out.numpy() if hasattr(out, "numpy") else np.asarray(out)
    assert np.allclose(out, ref(torch.from_numpy(x)).numpy(), atol=1e-5)


def test_ir_fake_quantize_and_group_conv(tmp_path):
    from zoo.pipeline.inference.openvino import load_openvino
    r = np.random.RandomState(2)
    wg = r.randn(4, 2, 1, 3, 3).astype(np.float32)   # 4 groups of 2 out / 1 in
    ir = _IR()
    x = ir.param([1, 4, 6, 6])
    lo, hi = ir.const(np.array(-1.0, np.float32)), ir.const(np.array(1.0, np.float32))
    q = ir.op("FakeQuantize", [x, lo, hi, lo, hi], {"levels": "256"})
    h = ir.op("GroupConvolution", [q, ir.const(wg)], {"strides": "1,1", "dilations": "1,1", "pads_begin": "1,1",
                                                       "pads_end": "1,1"})
    ir.result(ir.op("ReduceMean", [h, ir.const(np.array([2, 3], np.int64))], {"keep_dims": "false"}))
    m = load_openvino(*ir.save(str(tmp_path)))
    xt = torch.from_numpy(r.randn(1, 4, 6, 6).astype(np.float32))
    xq = torch.round((xt.clamp(-1, 1) + 1) / 2 * 255) / 255 * 2 - 1
    ref = F.conv2d(xq, torch.from_numpy(wg).reshape(8, 1, 3, 3), padding=1, groups=4).mean((2, 3))
    assert torch.allclose(m.predict(xt), ref, atol=1e-5)


def test_ir_v7_legacy_blobs(tmp_path):
    """IR v7: Input + layers with <blobs> (Convolution, ScaleShift, Pooling, FullyConnected)."""
    from zoo.pipeline.inference.openvino import load_openvino
    r = np.random.RandomState(3)
    w = r.randn(4, 3, 3, 3).astype(np.float32)
    b = r.randn(4).astype(np.float32)
    sc, sh = r.rand(4).astype(np.float32) + 0.5, r.randn(4).astype(np.float32)
    fw, fb = r.randn(3, 4 * 3 * 3).astype(np.float32), r.randn(3).astype(np.float32)
    blob = bytearray()

    def put(a):
        off = len(blob)
        blob.extend(a.tobytes())
        return off, a.nbytes
    (wo, ws), (bo, bs), (so, ss), (ho, hs), (fo, fs), (fbo, fbs) = map(put, (w, b, sc, sh, fw, fb))
    xml = f'''<?xml version="1.0"?><net name="v7" version="7" batch="1"><layers>
<layer id="0" name="data" type="Input" precision="FP32"><output><port id="0"><dim>1</dim><dim>3</dim><dim>6</dim><dim>6</dim></port></output></layer>
<layer id="1" name="conv" type="Convolution" precision="FP32"><data kernel="3,3" strides="1,1" pads_begin="1,1" pads_end="1,1" dilations="1,1" output="4" group="1"/>
<input><port id="0"/></input><output><port id="3"/></output><blobs><weights offset="{wo}" size="{ws}"/><biases offset="{bo}" size="{bs}"/></blobs></layer>
<layer id="2" name="ss" type="ScaleShift" precision="FP32"><input><port id="0"/></input><output><port id="3"/></output>
<blobs><weights offset="{so}" size="{ss}"/><biases offset="{ho}" size="{hs}"/></blobs></layer>
<layer id="3" name="relu" type="ReLU" precision="FP32"><input><port id="0"/></input><output><port id="1"/></output></layer>
<layer id="4" name="pool" type="Pooling" precision="FP32"><data kernel="2,2" strides="2,2" pads_begin="0,0" pads_end="0,0" pool-method="avg" exclude-pad="true"/>
<input><port id="0"/></input><output><port id="1"/></output></layer>
<layer id="5" name="fc" type="FullyConnected" precision="FP32"><data out-size="3"/><input><port id="0"/></input><output><port id="3"/></output>
<blobs><weights offset="{fo}" size="{fs}"/><biases offset="{fbo}" size="{fbs}"/></blobs></layer>
<layer id="6" name="prob" type="SoftMax" precision="FP32"><data axis="1"/><input><port id="0"/></input><output><port id="1"/></output></layer>
</layers><edges>
<edge from-layer="0" from-port="0" to-layer="1" to-port="0"/><edge from-layer="1" from-port="3" to-layer="2" to-port="0"/>
<edge from-layer="2" from-port="3" to-layer="3" to-port="0"/><edge from-layer="3" from-port="1" to-layer="4" to-port="0"/>
<edge from-layer="4" from-port="1" to-layer="5" to-port="0"/><edge from-layer="5" from-port="3" to-layer="6" to-port="0"/>
</edges></net>'''
    (tmp_path / "v7.xml").write_text(xml)
    (tmp_path / "v7.bin").write_bytes(bytes(blob))
    m = load_openvino(str(tmp_path / "v7.xml"))
    xt = torch.from_numpy(r.randn(1, 3, 6, 6).astype(np.float32))
    y = F.conv2d(xt, torch.from_numpy(w), torch.from_numpy(b), padding=1)
    y = F.relu(y * torch.from_numpy(sc).reshape(1, -1, 1, 1) + torch.from_numpy(sh).reshape(1, -1, 1, 1))
    y = F.avg_pool2d(y, 2, 2)
    ref = torch.softmax(F.linear(y.reshape(1, -1), torch.from_numpy(fw), torch.from_numpy(fb)), 1)
    assert torch.allclose(m.predict(xt), ref, atol=1e-5)


def test_ir_unsupported_layer_is_named(tmp_path):
    from zoo.pipeline.inference.openvino import load_openvino
    ir = _IR()
    x = ir.param([1, 4])
    ir.result(ir.op("ExperimentalDetectronROIFeatureExtractor", [x]))
    m = load_openvino(*ir.save(str(tmp_path)))
    with pytest.raises(NotImplementedError, match="ExperimentalDetectronROIFeatureExtractor"):
        m.predict(torch.zeros(1, 4))


@pytest.mark.gpu
def test_ir_v10_cnn_on_native_kernels(tmp_path):
    """On the GPU the IR's convolutions / matmul / max-pool run the native kernels (bf16
    MFMA): close to the fp32 CPU execution of the same IR."""
    from zoo.pipeline.inference.openvino import load_openvino
    r = np.random.RandomState(4)
    (xml, binp), ref = _cnn_ir(tmp_path, r)
    m = load_openvino(xml, binp).cuda()
    x = torch.from_numpy(r.randn(2, 3, 8, 8).astype(np.float32))
    out = m.predict(x.cuda()).float().cpu()
    assert len(m._native_w) == 2, "convolutions did not take the native path"
    assert (out - ref(x)).abs().max().item() < 2e-2
