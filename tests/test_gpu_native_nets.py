"""Every ImageClassifier backbone and both SSD detectors on the native NHWC kernels: per-layer
local parity (forward and backward) against the fp32 reference path, eval-mode end-to-end
logits, training through the engine; SSD loss and gradients against the fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

NETS = [("vgg-16", 224), ("alexnet", 227), ("squeezenet", 227), ("mobilenet", 224), ("mobilenet-v2", 224),
        ("inception-v1", 224), ("inception-v3", 299), ("densenet-161", 224)]


BANNED = ("miopen", "MIOpen", "mlo", "naive_conv", "gridwise_", "Cijk_")

def _layer_parity():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "analytics-zoo_amd",
                                    "tools"))
    import layer_parity
    return layer_parity


# Per-layer bounds (tools/layer_parity.py: the CPU twin computes with the bf16 weights the kernels
# read and rounds a conv output the GPU stores in bf16 before its BatchNorm, so a healthy layer
# differs only by accumulation order and output rounding). EVERY layer must meet them -- the
# reference KerasBaseSpec (zoo/src/test/scala/com/intel/analytics/zoo/pipeline/api/keras/layers/
# KerasBaseSpec.scala:45-90) checks every output and gradient, not a median. BatchNorm affine
# gradients are checked as the stacked [dgamma; dbeta] pair (dgamma alone is a cancelling sum).
# Measured r5 (profiles/r5/layer_parity_r5.md): every layer of the 8 backbones and both SSDs at
# <= 0.2 % forward, <= 0.33 % dx, <= 0.26 % weight gradients, <= 0.23 % BN affine; one conv's dgrad
# scaled by 1.05 shows 5.0 % in that layer alone
FWD_MAX = 0.01
DX_MAX = 0.01
DW_MAX = 0.01
AFFINE_MAX = 0.01
# (net, layer, metric) -> why the bound does not apply
EXEMPT = {}


def _violations(net, rows):
    bad = []
    for r in rows:
        checks = [("fwd", r["fwd"], FWD_MAX)]
        for k, v in r.items():
            if not isinstance(v, float) or not k.startswith("d"):
                continue
            if k == "dx":
                checks.append((k, v, DX_MAX))
            elif k == "daffine":
                checks.append((k, v, AFFINE_MAX))
            elif k not in ("dgamma", "dbeta"):
                checks.append((k, v, DW_MAX))
        for k, v, bound in checks:
            if v > bound and (net, r["layer"], k) not in EXEMPT:
                bad.append((r["layer"], k, v))
    return bad


def _calibrate_bn(model, x):
    """Running statistics = the batch statistics of ``x`` (one training forward at momentum 1):
    every BatchNorm then normalises in eval mode, so the eval network is numerically stable."""
    saved = {}
    for m in model.modules():
        if hasattr(m, "momentum") and hasattr(m, "running_mean"):
            saved[m] = m.momentum
            m.momentum = 1.0
    model.train()
    with torch.no_grad():
        model(x)
    for m, mom in saved.items():
        m.momentum = mom
    return model


@pytest.mark.parametrize("name,hw", NETS)
def test_backbone_layer_parity_and_trains_natively(gpu, name, hw, monkeypatch):
    """Every native layer against the SAME layer on the CPU path, fed the layer's actual GPU
    input and upstream gradient (tools/layer_parity.py): forward, dx, every weight gradient and
    the BatchNorm affine pair of EVERY layer within the per-layer bounds above (a wrong kernel
    shows O(1); the fault-injection test below shows a 5 % error in one layer fails). End to end
    in a stable regime -- eval mode with calibrated BatchNorm statistics -- the logits match the
    fp32 reference within 5 %. The GPU trace holds zoo:: kernels and no MIOpen / hipBLASLt kernel;
    then the engine trains the net (finite loss)."""
    import copy
    from torch.profiler import ProfilerActivity, profile
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image import native_nets
    from zoo.models.image.imageclassification.nets import build
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("nets-test")
    monkeypatch.setattr(native_nets, "_dropout", lambda x, p, training: x)
    torch.manual_seed(0)
    net = build(name, 16)
    cpu = copy.deepcopy(net)
    g = copy.deepcopy(net).to(gpu)
    x = torch.randn(2, 3, hw, hw)
    y = torch.randint(0, 16, (2,))
    lp = _layer_parity()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        rows = lp.run(g, cpu, x.to(gpu), lambda o: softmax_cross_entropy(o, y.to(gpu)), train=True)
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert any("zoo::" in n for n in names)
    bad = sorted({n for n in names if any(b in n for b in BANNED)})
    assert not bad, bad[:5]
    rows = [r for r in rows if "error" not in r]
    assert len(rows) >= 8, rows[:3]
    assert any("dx" in r for r in rows)
    bad = _violations(name, rows)
    print(name, "layers", len(rows), "max fwd", max(r["fwd"] for r in rows),
          "max dx", max(r.get("dx", 0.0) for r in rows), "violations", bad[:5])
    assert not bad, bad[:8]
    # end to end, stable regime: eval mode with calibrated BatchNorm statistics
    torch.manual_seed(1)
    net2 = build(name, 16)
    xc = torch.randn(8, 3, hw, hw)
    _calibrate_bn(net2, xc)
    g2 = copy.deepcopy(net2).to(gpu).eval()
    net2.eval()
    xe = torch.randn(4, 3, hw, hw)
    with torch.no_grad():
        lr = net2(xe).float()
        lg = g2(xe.to(gpu)).float().cpu()
    rel = ((lg - lr).norm() / lr.norm()).item()
    assert rel < 0.05, ("eval logits", rel)
    # and the engine trains it (fused optimizer, flat buffers)
    eng = TrainingEngine(build(name, 16), softmax_cross_entropy, SGD(learningrate=0.01, momentum=0.9))
    xg = torch.randn(4, 3, hw, hw, device=gpu)
    yg = torch.randint(0, 16, (4,), device=gpu)
    losses = [float(eng.train_step(xg, yg).item()) for _ in range(2)]
    assert all(l == l and 0 < l < 50 for l in losses), losses


def test_mobilenet_v2_matches_fp32_reference(gpu):
    """Eval-mode forward of the native net vs the same computation in fp32 torch (conv2d /
    depthwise groups=C / batch_norm with running stats)."""
    from zoo.models.image.native_nets import MobileNetV2, CBR, DWBR, _InvRes
    from zoo.models.image.resnet import Dense
    torch.manual_seed(0)
    m = MobileNetV2(16).to(gpu).eval()
    for mod in m.modules():  # non-trivial running statistics
        if hasattr(mod, "running_var"):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
    x = torch.randn(2, 3, 96, 96, device=gpu)

    def cbr(mod, h):
        R, S = mod.k
        C = h.shape[1]
        w = mod.weight[:, :R * S * (mod.weight.shape[1] // (R * S) if False else 0) or R * S * C]
        w = mod.weight[:, :R * S * C].reshape(-1, R, S, C).permute(0, 3, 1, 2)
        y = F.conv2d(h, w, stride=mod.stride, padding=mod.pad)
        y = F.batch_norm(y, mod.running_mean, mod.running_var, mod.gamma, mod.beta, False, 0.0, 1e-5)
        return y

    def dwbr(mod, h):
        C = h.shape[1]
        w = mod.weight.t().reshape(C, 1, *mod.k)
        y = F.conv2d(h, w, stride=mod.stride, padding=mod.pad, groups=C)
        y = F.batch_norm(y, mod.running_mean, mod.running_var, mod.gamma, mod.beta, False, 0.0, 1e-5)
        return torch.relu(y)

    with torch.no_grad():
        h = F.pad(x, (0, 0, 0, 0, 0, 1))  # 3 -> 4 input channels (zero)
        for layer in m.features:
            if isinstance(layer, CBR):
                h = torch.relu(cbr(layer, h)) if layer.relu else cbr(layer, h)
            else:
                inp = h
                if layer.expand is not None:
                    h = torch.relu(cbr(layer.expand, h))
                h = dwbr(layer.dw, h)
                h = cbr(layer.project, h)
                if layer.use_res:
                    h = h + inp
        h = h.mean((2, 3))
        ref = F.linear(h, m.fc.weight[:16], m.fc.bias[:16])
        out = m(x)
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel


@pytest.mark.parametrize("mobilenet", [False, True])
def test_ssd_trains_natively(gpu, mobilenet):
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "analytics-zoo_amd",
                                    "tools"))
    from zoo_models_bench import bench_ssd
    r = bench_ssd(2, 2, mobilenet=mobilenet)
    assert r["loss"] == r["loss"] and r["loss"] > 0


@pytest.mark.parametrize("mobilenet", [False, True])
def test_ssd_loss_and_gradient_parity(gpu, mobilenet):
    """SSD (VGG-16 / MobileNet, 300x300) on the native kernels vs the same weights on the fp32
    CPU path: MultiBoxLoss within 3 %, and per-layer local parity of EVERY layer of the
    detector (backbone, extras, loc / conf heads) in the training backward within the per-layer
    bounds above."""
    import copy
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.objectdetection.ssd import SSD, SSDMobileNet, MultiBoxLoss
    init_nncontext("ssd-parity")
    torch.manual_seed(0)
    model = SSDMobileNet(21) if mobilenet else SSD(21)
    crit = MultiBoxLoss(21)
    cpu = copy.deepcopy(model).train()
    g = copy.deepcopy(model).to(gpu).train()
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 300, 300)
    targets = []
    for _ in range(2):
        xy = torch.rand(3, 2, generator=gen) * 0.6
        wh = torch.rand(3, 2, generator=gen) * 0.3 + 0.05
        lab = torch.randint(1, 21, (3, 1), generator=gen).float()
        targets.append(torch.cat([lab, xy, xy + wh], 1))
    pri = model.priors
    oc = cpu(x)
    lc = float(crit(oc[0].float(), oc[1].float(), pri, targets))
    og = g(x.to(gpu))
    lg = float(crit(og[0].float(), og[1].float(), pri.to(gpu), [t.to(gpu) for t in targets]))
    assert abs(lg - lc) / abs(lc) < 0.03, (lg, lc)
    lp = _layer_parity()
    tg = [t.to(gpu) for t in targets]
    rows = lp.run(g, copy.deepcopy(model).train(), x.to(gpu),
                  lambda o: crit(o[0].float(), o[1].float(), pri.to(gpu), tg), train=True)
    rows = [r for r in rows if "error" not in r]
    assert len(rows) >= 10
    nm = "ssd-mobilenet" if mobilenet else "ssd-vgg"
    bad = _violations(nm, rows)
    print(nm, "loss", lg, lc, "max fwd", max(r["fwd"] for r in rows), "violations", bad[:5])
    assert not bad, bad[:8]


@pytest.mark.parametrize("name,hw", [("vgg-16", 224), ("mobilenet", 224)])
def test_layer_parity_catches_a_5pct_dgrad_fault(gpu, name, hw, monkeypatch):
    """ZOO_FAULT_DGRAD scales ONE conv's data gradient by 1.05 (zoo/ops/_kern.py): the per-layer
    check must flag exactly that kind of error (the median bar of r4 could not)."""
    import copy
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image import native_nets
    from zoo.models.image.imageclassification.nets import build
    from zoo.ops import _kern, softmax_cross_entropy
    init_nncontext("nets-fault")
    monkeypatch.setattr(native_nets, "_dropout", lambda x, p, training: x)
    torch.manual_seed(0)
    net = build(name, 16)
    x = torch.randn(2, 3, hw, hw)
    y = torch.randint(0, 16, (2,))
    lp = _layer_parity()
    monkeypatch.setenv("ZOO_FAULT_DGRAD", "3:1.05")
    _kern.reset_fault_counter()
    rows = lp.run(copy.deepcopy(net).to(gpu), copy.deepcopy(net), x.to(gpu),
                  lambda o: softmax_cross_entropy(o, y.to(gpu)), train=True)
    monkeypatch.delenv("ZOO_FAULT_DGRAD")
    bad = _violations(name, [r for r in rows if "error" not in r])
    assert bad and all(k == "dx" for _, k, _ in bad), bad
