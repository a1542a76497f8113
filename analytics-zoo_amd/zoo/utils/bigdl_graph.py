"""nn.Module models as BigDL ``nn`` graphs (VERDICT r2 missing #10; Topology.scala:708-825,
SURVEY.md §5.4).

The ResNet family (zoo.models.image.resnet: ConvBN units in NHWC with packed [K, R*S*C]
weights) is written as a BigDL ``StaticGraph`` of the standard modules a BigDL reader knows --
SpatialConvolution (NCHW weight [nGroup, out, in, kH, kW]), SpatialBatchNormalization
(gamma / beta + runningMean / runningVar), ReLU, CAddTable, SpatialMaxPooling,
SpatialAveragePooling (global), View and Linear -- instead of an opaque TorchModel blob. The
node names are the module paths, so the same file restores into a live model by name
(``restore_resnet``), and ``Net.load_bigdl`` (zoo.pipeline.api.net.bigdl_loader) rebuilds it as a
plain fp32 torch GraphNet that recomputes the forward.
"""
import numpy as np
import torch

BIGDL_NN = "com.intel.analytics.bigdl.nn."


class _Graph:
    def __init__(self):
        self.nodes = []          # spec dicts in topological order

    def add(self, kind, name, pre, attr=None, weight=None, bias=None):
        self.nodes.append({"type": BIGDL_NN + kind, "name": name, "attr": dict(attr or {}), "weight": weight,
                           "bias": bias, "pre": list(pre)})
        return name


def _np(t):
    return t.detach().float().cpu().numpy()


def _conv_bn(g, unit, path, x, cin_logical=None, resid=None):
    """ConvBN -> SpatialConvolution, SpatialBatchNormalization, (CAddTable), (ReLU)."""
    from zoo.ops.conv import unpack_weight
    K, k, C = unit.cout, unit.k, unit.cin
    w = unpack_weight(unit.weight.detach().float().cpu(), K, k, k, C)     # [K, R, S, C]
    if cin_logical is not None:
        w = w[..., :cin_logical]
        C = cin_logical
    w = w.permute(0, 3, 1, 2).reshape(1, K, C, k, k).numpy()
    conv = g.add("SpatialConvolution", path + "_conv", [] if x is None else [x],
                 {"nInputPlane": C, "nOutputPlane": K, "kernelW": k, "kernelH": k, "strideW": unit.stride,
                  "strideH": unit.stride, "padW": unit.pad, "padH": unit.pad, "nGroup": 1, "withBias": False,
                  "format": "NCHW"}, weight=w)
    bn = g.add("SpatialBatchNormalization", path + "_bn", [conv],
               {"nOutput": K, "eps": float(unit.eps), "momentum": float(unit.momentum), "affine": True,
                "runningMean": _np(unit.running_mean), "runningVar": _np(unit.running_var)},
               weight=_np(unit.gamma), bias=_np(unit.beta))
    out = bn
    if resid is not None:
        out = g.add("CAddTable", path + "_add", [bn, resid])
    if unit.relu:
        out = g.add("ReLU", path + "_relu", [out])
    return out


def resnet_graph_spec(model):
    """BigDL StaticGraph spec (dict for zoo.utils.bigdl_model._Writer) of a zoo ResNet."""
    from zoo.models.image.resnet import Bottleneck, BasicBlock
    g = _Graph()
    x = _conv_bn(g, model.stem, "stem", None, cin_logical=model.in_channels)
    x = g.add("SpatialMaxPooling", "stem_pool", [x], {"kW": 3, "kH": 3, "dW": 2, "dH": 2, "padW": 1, "padH": 1,
                                                      "ceilMode": False})
    for si, stage in enumerate(model.stages):
        for bi, blk in enumerate(stage):
            p = "stages.%d.%d" % (si, bi)
            sc = _conv_bn(g, blk.down, p + ".down", x) if blk.down is not None else x
            if isinstance(blk, Bottleneck):
                h = _conv_bn(g, blk.conv1, p + ".conv1", x)
                h = _conv_bn(g, blk.conv2, p + ".conv2", h)
                x = _conv_bn(g, blk.conv3, p + ".conv3", h, resid=sc)
            elif isinstance(blk, BasicBlock):
                h = _conv_bn(g, blk.conv1, p + ".conv1", x)
                x = _conv_bn(g, blk.conv2, p + ".conv2", h, resid=sc)
            else:
                raise TypeError("unsupported ResNet block %s" % type(blk).__name__)
    x = g.add("SpatialAveragePooling", "gap", [x], {"kW": 1, "kH": 1, "dW": 1, "dH": 1, "globalPooling": True})
    cin = model.fc.weight.shape[1]
    x = g.add("View", "flatten", [x], {"sizes": [cin], "numInputDims": 3})
    n = model.num_classes
    x = g.add("Linear", "fc", [x], {"inputSize": cin, "outputSize": n, "withBias": True},
              weight=_np(model.fc.weight[:n]), bias=_np(model.fc.bias[:n]))
    attr = {}
    for nd in g.nodes:
        attr[nd["name"] + "_edges"] = {"__edges__": nd["pre"], "name": nd["name"]}
    attr["inputNames"] = [g.nodes[0]["name"]]
    attr["outputNames"] = [x]
    attr["zoo_class"] = type(model).__module__ + "." + type(model).__qualname__
    attr["zoo_arch"] = {"blocks": [len(s) for s in model.stages], "block": type(model.stages[0][0]).__name__,
                        "width": int(model.stem.cout), "num_classes": int(n), "in_channels": int(model.in_channels)}
    attr["zoo_arch"] = str(attr["zoo_arch"])
    # the file lists nodes outputs-first (as BigDL's own graphs do)
    subs = [{k: v for k, v in nd.items()} for nd in reversed(g.nodes)]
    return {"type": BIGDL_NN + "StaticGraph", "name": type(model).__name__, "attr": attr, "submodules": subs}


def is_resnet(model):
    try:
        from zoo.models.image.resnet import ResNet
    except ImportError:  # pragma: no cover
        return False
    return isinstance(model, ResNet)


def restore_resnet(model, root, st):
    """Copy a BigDL ResNet graph's tensors into a live zoo ResNet by node name (layout
    conversion: NCHW conv weights -> packed NHWC [K, R*S*C], channels zero-padded)."""
    from zoo.ops.conv import pack_weight
    nodes = {s.name: s for s in root.submodules}

    def t(ref):
        return torch.from_numpy(ref.materialize(st).copy())

    def unit(path, u):
        cv, bn = nodes[path + "_conv"], nodes[path + "_bn"]
        K, k = u.cout, u.k
        w = t(cv.weight).reshape(K, -1, k, k).permute(0, 2, 3, 1)         # [K, R, S, Cin_logical]
        if w.shape[-1] != u.cin:
            w = torch.nn.functional.pad(w, (0, u.cin - w.shape[-1]))
        with torch.no_grad():
            u.weight.copy_(pack_weight(w).to(u.weight.dtype))
            u.gamma.copy_(t(bn.weight).reshape(-1))
            u.beta.copy_(t(bn.bias).reshape(-1))
            u.running_mean.copy_(torch.from_numpy(bn.attr["runningMean"].materialize(st)).reshape(-1))
            u.running_var.copy_(torch.from_numpy(bn.attr["runningVar"].materialize(st)).reshape(-1))

    unit("stem", model.stem)
    for si, stage in enumerate(model.stages):
        for bi, blk in enumerate(stage):
            p = "stages.%d.%d" % (si, bi)
            for nm in ("conv1", "conv2", "conv3", "down"):
                u = getattr(blk, nm, None)
                if u is not None:
                    unit(p + "." + nm, u)
    fc = nodes["fc"]
    n = model.num_classes
    with torch.no_grad():
        model.fc.weight.zero_()
        model.fc.bias.zero_()
        model.fc.weight[:n].copy_(t(fc.weight).reshape(n, -1))
        model.fc.bias[:n].copy_(t(fc.bias).reshape(-1))
    return model


def nchw_input(x):
    """NCHW input for the decoded graph (the zoo ResNet takes NCHW images too)."""
    return x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
