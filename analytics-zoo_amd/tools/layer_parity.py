#!/usr/bin/env python3
"""Per-layer LOCAL parity of a native NHWC network against its CPU fp32 reference path.

For every leaf module of the GPU model the forward hook records the module's actual GPU input
(and the backward hook its upstream gradient); the SAME module of a CPU copy (same weights) is
then run on exactly those inputs in fp32 and compared. Unlike an end-to-end comparison this
isolates each kernel from the rounding noise that the layers before it accumulate: a healthy
bf16 layer shows ~0.2-1 % local error, a wrong kernel shows O(1).

  python tools/layer_parity.py --net mobilenet [--hw 224] [--batch 2] [--out f.json]
  python tools/layer_parity.py --frcnn pvanet
"""
import argparse
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def _rel(a, b):
    a, b = a.detach().float().cpu().flatten(), b.detach().float().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-20))


def _leaves(m):
    out = []
    for name, mod in m.named_modules():
        if not list(mod.children()) or any(True for _ in mod.parameters(recurse=False)):
            if name:
                out.append((name, mod))
    return out


def _tensors(xs):
    return [x for x in (xs if isinstance(xs, (list, tuple)) else [xs]) if torch.is_tensor(x)]


def _round_weights_bf16(cmodel):
    """The CPU twin computes with the bf16 values the GPU kernels read for matrix weights (dim >= 2:
    packed conv / dense / depthwise weights); BatchNorm affine and biases stay fp32 as on the GPU.
    Without it the per-weight bf16 rounding alone moves pre-activations across ReLU's zero in
    ~0.1 % of the elements, a ~3-4 % L2 difference in dx that would mask real kernel errors."""
    with torch.no_grad():
        for p in cmodel.parameters():
            if p.dim() >= 2:
                p.copy_(p.to(torch.bfloat16).float())


def affine_rel(row):
    """BatchNorm affine gradients relative to the norm of the stacked [dgamma; dbeta] reference:
    dgamma is a cancelling sum (sum dy * xhat: exactly zero at gamma=1, beta=0 for a unit whose
    consumer normalises again, e.g. conv-BN-ReLU -> depthwise-BN), so its own norm is no scale."""
    return row.get("daffine")


def run(gmodel, cmodel, x, loss_fn, train=True, round_bf16=True):
    gmodel.train(train)
    cmodel.train(train)
    if round_bf16:
        _round_weights_bf16(cmodel)
    cmods = dict(_leaves(cmodel))
    rec = {}
    hooks = []
    order = []
    for name, mod in _leaves(gmodel):
        def fwd(mod, inp, kw, out, name=name):
            if name not in rec:
                order.append(name)
                # keyword tensors too (e.g. a fused residual, ``unit(x, resid=r)``): the CPU twin
                # must see the same inputs or a fused add reads as an O(1) forward error
                kwt = {k: v.detach().clone() for k, v in (kw or {}).items() if torch.is_tensor(v)}
                rec[name] = {"in": [t.detach().clone() for t in _tensors(inp)], "kw": kwt,
                             "out": [t.detach().clone() for t in _tensors(out)]}
        hooks.append(mod.register_forward_hook(fwd, with_kwargs=True))

        def bwd(mod, gin, gout, name=name):
            if name in rec and "gout" not in rec[name]:
                rec[name]["gout"] = [None if g is None else g.detach().clone() for g in gout]
                rec[name]["gin"] = [None if g is None else g.detach().clone() for g in gin]
        hooks.append(mod.register_full_backward_hook(bwd))
    out = gmodel(x)
    if train:
        loss_fn(out).backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    gparams = {n: p for n, p in gmodel.named_parameters()}
    rows = []
    from zoo.ops.conv import REF_BF16_STORAGE
    saved = REF_BF16_STORAGE[0]
    REF_BF16_STORAGE[0] = bool(round_bf16)
    try:
        _compare(order, rec, cmods, gparams, rows, train)
    finally:
        REF_BF16_STORAGE[0] = saved
    return rows


def _tie_masked(cm, r, xs, kws, y_ref, row):
    """Re-run the CPU twin with its ReLU keeping exactly the elements the GPU forward kept
    (zoo.ops.conv.REF_RELU_MASK) when the two forwards disagree on some element's sign: such an
    element sits within rounding of zero (the forward metric already bounds the outputs), and
    the backward comparison should not charge its whole gradient to the kernels. Applies only
    when the module ran exactly one ReLU of the output's shape; ``row["ties"]`` counts them."""
    from zoo.ops.conv import REF_RELU_MASK
    out = r["out"][0].float().cpu()
    if out.shape != y_ref.shape or out.min() < 0:
        return None
    keep = out > 0
    ties = int((keep != (y_ref.detach() > 0)).sum())
    if ties == 0:
        return None
    xs2 = [t.detach().clone().requires_grad_(t.is_floating_point()) for t in xs]
    for p in cm.parameters():
        p.grad = None
    REF_RELU_MASK[0], REF_RELU_MASK[1] = keep, 0
    try:
        y2 = cm(*xs2, **kws)
        uses = REF_RELU_MASK[1]
    finally:
        REF_RELU_MASK[0], REF_RELU_MASK[1] = None, 0
    if uses != 1:
        for p in cm.parameters():
            p.grad = None
        return None
    row["ties"] = ties
    return xs2, _tensors(y2)


def _compare(order, rec, cmods, gparams, rows, train):
    for name in order:
        r = rec[name]
        cm = cmods.get(name)
        if cm is None or not r["in"]:
            continue
        xs = [t.float().cpu().requires_grad_(t.is_floating_point()) for t in r["in"]]
        for p in cm.parameters():
            p.grad = None
        kws = {k: v.float().cpu() for k, v in (r["kw"] or {}).items()}
        try:
            y = cm(*xs, **kws)
        except Exception as e:  # noqa: BLE001
            rows.append({"layer": name, "type": type(cm).__name__, "error": str(e)[:200]})
            continue
        ys = _tensors(y)
        row = {"layer": name, "type": type(cm).__name__, "shape": list(r["out"][0].shape),
               "fwd": round(_rel(r["out"][0], ys[0]), 5)}
        if train and "gout" in r and r["gout"][0] is not None:
            gy = r["gout"][0].float().cpu()
            masked = _tie_masked(cm, r, xs, kws, ys[0], row)
            if masked is not None:
                xs, ys = masked
            if gy.shape == ys[0].shape:
                ys[0].backward(gy)
                gins = [g for g in r["gin"]]
                if gins and gins[0] is not None and xs[0].grad is not None:
                    row["dx"] = round(_rel(gins[0], xs[0].grad), 5)
                for pn, p in cm.named_parameters(recurse=False):
                    gp = gparams.get(name + "." + pn)
                    if p.grad is not None and gp is not None and gp.grad is not None and p.grad.abs().max() > 0:
                        row["d" + pn] = round(_rel(gp.grad, p.grad), 5)
                # BatchNorm affine pair, normalised by the pair's reference norm (affine_rel)
                pair = [(name + "." + a, getattr(cm, a, None)) for a in ("gamma", "beta")]
                if all(isinstance(q, torch.Tensor) and q.grad is not None and gparams.get(n) is not None and
                       gparams[n].grad is not None for n, q in pair):
                    ref = torch.cat([q.grad.flatten() for _, q in pair])
                    got = torch.cat([gparams[n].grad.detach().float().cpu().flatten() for n, _ in pair])
                    row["daffine"] = round(_rel(got, ref), 5)
        rows.append(row)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", default=None)
    ap.add_argument("--frcnn", default=None)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--eval", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    if a.net:
        from zoo.models.image import native_nets
        from zoo.models.image.imageclassification.nets import build
        native_nets._dropout = lambda x, p, training: x
        net = build(a.net, 16)
        cpu = copy.deepcopy(net)
        g = copy.deepcopy(net).to(dev)
        x = torch.randn(a.batch, 3, a.hw, a.hw, device=dev)
        y = torch.randint(0, 16, (a.batch,), device=dev)
        from zoo.ops import softmax_cross_entropy
        rows = run(g, cpu, x, lambda o: softmax_cross_entropy(o, y), train=not a.eval)
    else:
        from zoo.models.image.objectdetection.frcnn import FasterRCNN
        m = FasterRCNN(num_classes=21, backbone=a.frcnn, pre_nms_topn=600, post_nms_topn=50).eval()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Conv2d):
                torch.nn.init.normal_(mod.weight, 0, (2.0 / (mod.in_channels * mod.kernel_size[0] ** 2)) ** 0.5)
        cpu = copy.deepcopy(m)
        g = copy.deepcopy(m).to(dev)
        x = torch.randn(1, 3, 224, 320, device=dev)

        class _F(torch.nn.Module):
            def __init__(self, mm):
                super().__init__()
                self.mm = mm

            def forward(self, z):
                return self.mm.features_nhwc(z) if z.is_cuda else self.mm.features(z)
        with torch.no_grad():
            rows = run(_F(g), _F(cpu), x, None, train=False)
    for r in rows:
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
