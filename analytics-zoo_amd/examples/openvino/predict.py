#!/usr/bin/env python3
"""OpenVINO IR inference (pyzoo/zoo/examples/openvino/predict.py): an IR (xml + bin) is loaded
with InferenceModel.load_openvino -- decoded and executed by this framework, convolutions and
matmuls on the native kernels -- and run on a batch. Without --xml a small IR v10 CNN is written
first (the same layer set an exported classification network uses)."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def write_ir(d, rng, classes=5):
    """A Conv-ReLU-Pool-Conv-GAP-MatMul-SoftMax IR v10 network; returns (xml, bin)."""
    layers, edges, blob = [], [], bytearray()

    def add(xml_fmt, *args):
        i = len(layers)
        layers.append(xml_fmt % ((i, i) + args))
        return i

    def const(arr):
        arr = np.ascontiguousarray(arr, np.float32)
        off = len(blob)
        blob.extend(arr.tobytes())
        dims = "".join("<dim>%d</dim>" % v for v in arr.shape)
        return add('<layer id="%d" name="c%d" type="Const" version="opset1"><data element_type="f32" shape="%s" '
                   'offset="%d" size="%d"/><output><port id="0">%s</port></output></layer>',
                   ",".join(map(str, arr.shape)), off, arr.nbytes, dims)

    def op(typ, ins, attrs=""):
        i = add('<layer id="%d" name="n%d" type="' + typ + '" version="opset1">' + (attrs and "<data %s/>" % attrs)
                + "<input>" + "".join('<port id="%d"/>' % k for k in range(len(ins))) + "</input>"
                + '<output><port id="%d"/></output></layer>' % len(ins))
        for k, src in enumerate(ins):
            edges.append('<edge from-layer="%d" from-port="%d" to-layer="%d" to-port="%d"/>'
                         % (src, 0 if layers[src].find('type="Parameter"') >= 0 or 'type="Const"' in layers[src]
                            else layers[src].count('<port id=') - 1, i, k))
        return i
    x = add('<layer id="%d" name="in%d" type="Parameter" version="opset1"><data shape="1,3,32,32" element_type="f32"/>'
            '<output><port id="0"><dim>1</dim><dim>3</dim><dim>32</dim><dim>32</dim></port></output></layer>')
    conv = 'strides="1,1" dilations="1,1" pads_begin="1,1" pads_end="1,1" auto_pad="explicit"'
    h = op("Convolution", [x, const(rng.standard_normal((8, 3, 3, 3)) * 0.3)], conv)
    h = op("Relu", [h])
    h = op("MaxPool", [h], 'strides="2,2" kernel="2,2" pads_begin="0,0" pads_end="0,0" rounding_type="floor"')
    h = op("Convolution", [h, const(rng.standard_normal((16, 8, 3, 3)) * 0.2)], conv)
    h = op("ReduceMean", [h, add('<layer id="%d" name="ax%d" type="Const" version="opset1"><data element_type="i64" '
                                 'shape="2" offset="%d" size="16"/><output><port id="0"><dim>2</dim></port></output>'
                                 '</layer>', len(blob))], 'keep_dims="false"')
    blob.extend(np.array([2, 3], np.int64).tobytes())
    h = op("MatMul", [h, const(rng.standard_normal((classes, 16)) * 0.3)], 'transpose_a="false" transpose_b="true"')
    h = op("SoftMax", [h], 'axis="1"')
    r = add('<layer id="%d" name="out%d" type="Result" version="opset1"><input><port id="0"/></input></layer>')
    edges.append('<edge from-layer="%d" from-port="1" to-layer="%d" to-port="0"/>' % (h, r))
    xml = os.path.join(d, "model.xml")
    with open(xml, "w") as f:
        f.write('<?xml version="1.0"?><net name="example" version="10"><layers>%s</layers><edges>%s</edges></net>'
                % ("".join(layers), "".join(edges)))
    with open(os.path.join(d, "model.bin"), "wb") as f:
        f.write(bytes(blob))
    return xml, os.path.join(d, "model.bin")


def main(argv=None):
    ap = _common.add_common(argparse.ArgumentParser(description=__doc__.split("\n")[0]))
    ap.add_argument("--xml", default=None)
    ap.add_argument("--bin", default=None)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args(argv)
    from zoo.pipeline.inference import InferenceModel
    rng = np.random.default_rng(a.seed)
    with tempfile.TemporaryDirectory() as d:
        xml, binp = (a.xml, a.bin) if a.xml else write_ir(d, rng)
        im = InferenceModel(1).load_openvino(xml, binp)
        x = rng.standard_normal((a.batch, 3, 32, 32)).astype(np.float32)
        out = np.asarray(im.predict(x))
    print("predictions", out.argmax(-1).tolist(), "rows sum to", np.round(out.sum(-1), 4).tolist())
    return out


if __name__ == "__main__":
    main()
