"""nn.Module models as BigDL ``nn`` graphs (VERDICT r2 missing #10; Topology.scala:708-825,
SURVEY.md §5.4). ResNet is written from its block structure; the other native ImageClassifier
backbones (ImageClassificationConfig.scala:56-190) by tracing one CPU forward (native_graph_spec).

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


# ---------------------------------------------------------------------------------------------
# native ImageClassifier backbones (zoo.models.image.native_nets): traced, not hand-listed
#
# The nets' forwards mix units (CBR / CB / DWBR / BNR / pools / Dense) with a little functional
# glue (channel concat, ReLU, residual add, flatten, dropout, class slicing). One CPU forward of
# the model at its native input size is recorded: forward hooks turn each unit call into BigDL
# modules (NHWC packed weights -> NCHW layouts), a TorchFunctionMode records the glue between
# units (and refuses anything it cannot express, so an unknown graph never silently loses an op).

_GLUE_ALIAS = ("float", "to", "contiguous", "bfloat16", "clone", "detach")


class _NetTracer:
    def __init__(self, model):
        from zoo.models.image import native_nets as nn_
        self.nn = nn_
        self.model = model
        self.g = _Graph()
        self.names = {}          # id(tensor) -> node name
        self.meta = {}           # node name -> {"cin": logical channels} / {"flat": (H, W, C)}
        self.keep = []           # keeps traced tensors alive (stable ids)
        self.depth = 0
        self.paths = {id(m): p for p, m in model.named_modules()}
        self.count = {}

    # -------------------------------------------------------------------- bookkeeping
    def _name(self, base):
        base = base or "node"
        k = self.count.get(base, 0)
        self.count[base] = k + 1
        return base if k == 0 else "%s#%d" % (base, k)

    def bind(self, t, name, meta=None):
        self.names[id(t)] = name
        self.keep.append(t)
        if meta:
            self.meta[name] = meta

    def src(self, t):
        if id(t) not in self.names:
            raise NotImplementedError("traced tensor of unknown origin (shape %s)" % (tuple(t.shape),))
        return self.names[id(t)]

    # -------------------------------------------------------------------- units
    def unit(self, mod, args, kwargs, out):
        nn_ = self.nn
        from zoo.models.image.resnet import Dense
        from zoo.ops.conv import unpack_weight
        path = self.paths.get(id(mod), type(mod).__name__)
        x = args[0]
        pre = self.src(x)
        cin_log = self.meta.get(pre, {}).get("cin")
        g = self.g
        base = self._name(path)
        if isinstance(mod, (nn_.CBR, nn_.CB)):
            R, S = mod.k
            C = x.shape[-1]
            K = mod.weight.shape[0]
            w = unpack_weight(mod.weight.detach().float().cpu(), K, R, S, C)
            bias = None
            if isinstance(mod, nn_.CB):
                w, bias = w[:mod.cout], _np(mod.bias[:mod.cout])
                K = mod.cout
            if cin_log is not None:
                w, C = w[..., :cin_log], cin_log
            w = w.permute(0, 3, 1, 2).reshape(1, K, C, R, S).numpy()
            attr = {"nInputPlane": C, "nOutputPlane": K, "kernelW": S, "kernelH": R, "strideW": mod.stride[1],
                    "strideH": mod.stride[0], "padW": mod.pad[1], "padH": mod.pad[0], "nGroup": 1,
                    "withBias": bias is not None, "format": "NCHW"}
            if isinstance(mod, nn_.CB) and tuple(mod.dil) != (1, 1):
                attr.update({"dilationW": mod.dil[1], "dilationH": mod.dil[0]})
            attr["zoo_cin"] = int(x.shape[-1])          # the unit's (padded) NHWC input channels
            kind = "SpatialDilatedConvolution" if "dilationW" in attr else "SpatialConvolution"
            y = g.add(kind, base + "_conv", [pre], attr, weight=w, bias=bias)
            if isinstance(mod, nn_.CBR):
                y = self._bn(base, y, mod, K)
                resid = kwargs.get("resid", args[1] if len(args) > 1 else None)
                if resid is not None:
                    y = g.add("CAddTable", base + "_add", [y, self.src(resid)])
            elif mod.relu:
                y = g.add("ReLU", base + "_relu", [y])
        elif isinstance(mod, nn_.DWBR):
            R, S = mod.k
            C = mod.weight.shape[1]
            w = mod.weight.detach().float().cpu().t().reshape(C, 1, 1, R, S).numpy()
            y = g.add("SpatialConvolution", base + "_conv", [pre],
                      {"nInputPlane": C, "nOutputPlane": C, "kernelW": S, "kernelH": R, "strideW": mod.stride[1],
                       "strideH": mod.stride[0], "padW": mod.pad[1], "padH": mod.pad[0], "nGroup": C,
                       "withBias": False, "format": "NCHW"}, weight=w)
            y = self._bn(base, y, mod, C)
        elif isinstance(mod, nn_.BNR):
            y = self._bn(base, pre, mod, mod.gamma.shape[0])
        elif isinstance(mod, nn_.MaxPool):
            y = g.add("SpatialMaxPooling", base + "_pool", [pre],
                      {"kW": mod.k[1], "kH": mod.k[0], "dW": mod.s[1], "dH": mod.s[0], "padW": mod.p[1],
                       "padH": mod.p[0], "ceilMode": bool(mod.ceil)})
        elif isinstance(mod, nn_.AvgPool):
            y = g.add("SpatialAveragePooling", base + "_pool", [pre],
                      {"kW": mod.k[1], "kH": mod.k[0], "dW": mod.s[1], "dH": mod.s[0], "padW": mod.p[1],
                       "padH": mod.p[0], "ceilMode": bool(mod.ceil), "countIncludePad": bool(mod.inc)})
        elif isinstance(mod, Dense):
            n = mod.cout
            w = mod.weight.detach().float().cpu()[:n]
            flat = self.meta.get(pre, {}).get("flat")
            lattr = {"inputSize": int(w.shape[1]), "outputSize": n, "withBias": True}
            if flat is not None:           # NHWC flatten in the native net, NCHW flatten in BigDL
                H, W, C = flat
                w = w.reshape(n, H, W, C).permute(0, 3, 1, 2).reshape(n, -1)
                lattr["zoo_nhwc_flat"] = [int(H), int(W), int(C)]
            y = g.add("Linear", base + "_linear", [pre], lattr, weight=w.numpy(), bias=_np(mod.bias[:n]))
        else:
            raise NotImplementedError(type(mod).__name__)
        self.bind(out, y)

    def _bn(self, base, pre, mod, c):
        y = self.g.add("SpatialBatchNormalization", base + "_bn", [pre],
                       {"nOutput": int(c), "eps": 1e-5, "momentum": 0.1, "affine": True,
                        "runningMean": _np(mod.running_mean), "runningVar": _np(mod.running_var)},
                       weight=_np(mod.gamma), bias=_np(mod.beta))
        if mod.relu:
            y = self.g.add("ReLU", base + "_relu", [y])
        return y

    # -------------------------------------------------------------------- glue
    def glue(self, func, args, kwargs, out):
        """Record one functional op between units; returns True when handled."""
        name = getattr(func, "__name__", str(func))
        tens = [a for a in args if isinstance(a, torch.Tensor) and id(a) in self.names]
        if not isinstance(out, torch.Tensor) or not tens:
            return
        g = self.g
        x = tens[0]
        pre = self.src(x)
        if name in _GLUE_ALIAS:
            self.bind(out, pre, self.meta.get(pre))
        elif name in ("relu", "relu_"):
            self.bind(out, g.add("ReLU", self._name("relu"), [pre]))
        elif name in ("add", "__add__", "__radd__"):
            ts = [a for a in args if isinstance(a, torch.Tensor)]
            if len(ts) != 2 or any(id(t) not in self.names for t in ts):
                raise NotImplementedError("add of a non-traced operand")
            self.bind(out, g.add("CAddTable", self._name("add"), [self.src(t) for t in ts]))
        elif name in ("reshape", "view", "flatten") and x.dim() == 4 and out.dim() == 2:
            nm = g.add("View", self._name("flatten"), [pre], {"sizes": [int(out.shape[1])], "numInputDims": 3})
            self.bind(out, nm, {"flat": tuple(int(v) for v in x.shape[1:])})
        elif name == "__getitem__" and x.dim() == 2 and out.dim() == 2 and out.shape[0] == x.shape[0]:
            n = int(out.shape[1])
            if n == x.shape[1]:
                self.bind(out, pre)
            else:
                idx = args[1]
                if not (isinstance(idx, tuple) and len(idx) == 2 and isinstance(idx[1], slice) and
                        idx[1].start in (None, 0) and idx[1].step in (None, 1)):
                    raise NotImplementedError("unsupported slice %r" % (idx,))
                self.bind(out, g.add("Narrow", self._name("narrow"), [pre],
                                     {"dimension": 2, "offset": 1, "length": n}))
        else:
            raise NotImplementedError("op %s between units is not expressible as a BigDL module" % name)

    # -------------------------------------------------------------------- functional helpers
    def f_prepare(self, x, *a, **k):
        return x

    def f_gap(self, x):
        y = x.float().mean(dim=(1, 2)).to(x.dtype)
        p = self.g.add("SpatialAveragePooling", self._name("gap"), [self.src(x)],
                       {"kW": 1, "kH": 1, "dW": 1, "dH": 1, "globalPooling": True})
        self.bind(y, self.g.add("View", self._name("gap_flatten"), [p],
                                {"sizes": [int(x.shape[-1])], "numInputDims": 3}))
        return y

    def f_cat(self, xs):
        y = torch.cat(xs, dim=-1)
        self.bind(y, self.g.add("JoinTable", self._name("concat"), [self.src(t) for t in xs],
                                {"dimension": 1, "nInputDims": 3}))
        return y

    def f_dropout(self, x, p, training):
        y = x.clone()
        pre = self.src(x)
        self.bind(y, self.g.add("Dropout", self._name("dropout"), [pre], {"initP": float(p)}), self.meta.get(pre))
        return y


def native_graph_spec(model, hw=None):
    """BigDL StaticGraph spec of a native ImageClassifier backbone (one traced CPU forward)."""
    import copy
    from torch.overrides import TorchFunctionMode
    from zoo.models.image import native_nets as nn_
    from zoo.models.image.resnet import Dense
    src = copy.deepcopy(model).cpu().float().eval()
    tr = _NetTracer(src)
    units = (nn_.CBR, nn_.CB, nn_.DWBR, nn_.BNR, nn_.MaxPool, nn_.AvgPool, Dense)
    handles = []

    def pre_hook(mod, args, kwargs):
        tr.depth += 1

    def post_hook(mod, args, kwargs, out):
        tr.depth -= 1
        if tr.depth == 0:
            tr.unit(mod, args, kwargs, out)
        return out
    for m in src.modules():
        if isinstance(m, units):
            handles.append(m.register_forward_pre_hook(pre_hook, with_kwargs=True))
            handles.append(m.register_forward_hook(post_hook, with_kwargs=True))

    class Glue(TorchFunctionMode):
        def __torch_function__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            out = func(*args, **kwargs)
            if tr.depth == 0:
                tr.glue(func, args, kwargs, out)
            return out

    def wrap(fn):
        def w(*a, **k):
            tr.depth += 1
            try:
                return fn(*a, **k)
            finally:
                tr.depth -= 1
        return w
    saved = {k: getattr(nn_, k) for k in ("gap", "cat", "_dropout")}
    hw = hw or getattr(model, "trace_hw", 224)
    x = torch.zeros(1, src.in_channels, hw, hw)
    xin = src.prepare(x)
    tr.bind(xin, tr.g.add("Input", "input", []), {"cin": src.in_channels})
    try:
        nn_.gap, nn_.cat, nn_._dropout = wrap(tr.f_gap), wrap(tr.f_cat), wrap(tr.f_dropout)
        src.prepare = lambda t: t                       # the traced input is already prepared
        with torch.no_grad(), Glue():
            out = src(xin)
    finally:
        for k, v in saved.items():
            setattr(nn_, k, v)
        for h in handles:
            h.remove()
    g = tr.g
    attr = {}
    for nd in g.nodes:
        attr[nd["name"] + "_edges"] = {"__edges__": nd["pre"], "name": nd["name"]}
    attr["inputNames"] = ["input"]
    attr["outputNames"] = [tr.src(out)]
    attr["zoo_class"] = type(model).__module__ + "." + type(model).__qualname__
    attr["zoo_input_hw"] = int(hw)
    subs = [{k: v for k, v in nd.items()} for nd in reversed(g.nodes)]
    return {"type": BIGDL_NN + "StaticGraph", "name": type(model).__name__, "attr": attr, "submodules": subs}


def is_native_net(model):
    try:
        from zoo.models.image.native_nets import NativeNet
    except ImportError:  # pragma: no cover
        return False
    return isinstance(model, NativeNet)


def restore_native(model, root, st):
    """Copy a traced native-net graph's tensors back into a live net by module path (inverse of
    the layout conversions in _NetTracer.unit)."""
    from zoo.models.image import native_nets as nn_
    from zoo.models.image.resnet import Dense
    from zoo.ops.conv import pack_weight
    nodes = {s.name: s for s in root.submodules}

    def t(ref):
        return torch.from_numpy(ref.materialize(st).copy())

    def arr(v):
        return torch.from_numpy(np.asarray(v.materialize(st)).copy()).reshape(-1)

    def bn(base, mod):
        b = nodes[base + "_bn"]
        mod.gamma.copy_(t(b.weight).reshape(-1))
        mod.beta.copy_(t(b.bias).reshape(-1))
        mod.running_mean.copy_(arr(b.attr["runningMean"]))
        mod.running_var.copy_(arr(b.attr["runningVar"]))

    with torch.no_grad():
        for path, mod in model.named_modules():
            if isinstance(mod, (nn_.CBR, nn_.CB)):
                cv = nodes[path + "_conv"]
                R, S = mod.k
                a = cv.attr
                C_log, Kl, cin = int(a["nInputPlane"]), int(a["nOutputPlane"]), int(a["zoo_cin"])
                w = t(cv.weight).reshape(Kl, C_log, R, S).permute(0, 2, 3, 1)    # [K, R, S, C]
                w4 = torch.zeros(mod.weight.shape[0], R, S, cin)
                w4[:Kl, :, :, :C_log] = w
                mod.weight.copy_(pack_weight(w4).to(mod.weight.dtype))
                if isinstance(mod, nn_.CB):
                    mod.bias.zero_()
                    mod.bias[:Kl].copy_(t(cv.bias).reshape(-1))
                else:
                    bn(path, mod)
            elif isinstance(mod, nn_.DWBR):
                C = mod.weight.shape[1]
                mod.weight.copy_(t(nodes[path + "_conv"].weight).reshape(C, -1).t())
                bn(path, mod)
            elif isinstance(mod, nn_.BNR):
                bn(path, mod)
            elif isinstance(mod, Dense):
                lin = nodes[path + "_linear"]
                n = mod.cout
                w = t(lin.weight).reshape(n, -1)
                flat = lin.attr.get("zoo_nhwc_flat")
                if flat:
                    H, W, C = (int(v) for v in flat)
                    w = w.reshape(n, C, H, W).permute(0, 2, 3, 1).reshape(n, -1)
                mod.weight.zero_()
                mod.bias.zero_()
                mod.weight[:n].copy_(w)
                mod.bias[:n].copy_(t(lin.bias).reshape(-1))
    return model
