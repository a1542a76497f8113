"""ResNet-50 bench-config parity: the native bf16 training step vs a plain
PyTorch fp32 ResNet-50 (F.conv2d / F.batch_norm / torch.optim.SGD) started
from the SAME weights on the SAME batch.

  python tools/resnet_parity.py [--batch 256] [--steps 30] [--lr 0.1] [--warmup-steps 0]

Prints (1) per-parameter-group gradient cosine / relative-norm of the first
step, (2) the loss trajectories of both runs side by side, and (3) with
``--repeat`` the native trajectory of a second identical-seed run (to expose
run-to-run non-determinism). Reference run: the BigDL TrainImageNet example
(Zs/examples/resnet/TrainImageNet.scala) trains the same network with
SGD(momentum 0.9, wd 1e-4) and an EpochDecayWithWarmUp schedule.
"""
import argparse
import copy
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402


class RefConvBN(nn.Module):
    def __init__(self, zc, cin_real=None):
        super().__init__()
        K, R, C = zc.cout, zc.k, zc.cin
        w4 = zc.weight.detach()[:, :R * R * C].reshape(K, R, R, C).float()
        if cin_real is not None:
            w4 = w4[..., :cin_real]
        self.weight = nn.Parameter(w4.permute(0, 3, 1, 2).contiguous())
        self.gamma = nn.Parameter(zc.gamma.detach().float().clone())
        self.beta = nn.Parameter(zc.beta.detach().float().clone())
        self.register_buffer("rm", zc.running_mean.detach().float().clone())
        self.register_buffer("rv", zc.running_var.detach().float().clone())
        self.stride, self.pad, self.relu, self.eps, self.mom = zc.stride, zc.pad, zc.relu, zc.eps, zc.momentum

    def forward(self, x, resid=None):
        y = F.conv2d(x, self.weight, stride=self.stride, padding=self.pad)
        y = F.batch_norm(y, self.rm, self.rv, self.gamma, self.beta, self.training, self.mom, self.eps)
        if resid is not None:
            y = y + resid
        return torch.relu(y) if self.relu else y


class RefBottleneck(nn.Module):
    def __init__(self, zb):
        super().__init__()
        self.conv1, self.conv2, self.conv3 = RefConvBN(zb.conv1), RefConvBN(zb.conv2), RefConvBN(zb.conv3)
        self.down = RefConvBN(zb.down) if zb.down is not None else None

    def forward(self, x):
        sc = self.down(x) if self.down is not None else x
        return self.conv3(self.conv2(self.conv1(x)), resid=sc)


class RefResNet(nn.Module):
    """fp32 NCHW twin of zoo.models.image.resnet.ResNet (Bottleneck only)."""

    def __init__(self, zm):
        super().__init__()
        self.stem = RefConvBN(zm.stem, cin_real=zm.in_channels)
        self.stages = nn.Sequential(*[nn.Sequential(*[RefBottleneck(b) for b in st]) for st in zm.stages])
        nc = zm.num_classes
        self.fc_w = nn.Parameter(zm.fc.weight.detach()[:nc].float().clone())
        self.fc_b = nn.Parameter(zm.fc.bias.detach()[:nc].float().clone())

    def forward(self, x):
        x = self.stem(x)
        x = F.max_pool2d(x, 3, 2, 1)
        x = self.stages(x)
        x = x.mean((2, 3))
        return F.linear(x, self.fc_w, self.fc_b)


def zoo_grad_views(zm):
    """name -> (zoo grad tensor as the ref layout, ref param name)."""
    out = {}
    for name, mod in zm.named_modules():
        if hasattr(mod, "gamma") and hasattr(mod, "k"):
            K, R, C = mod.cout, mod.k, mod.cin
            g = mod.weight.grad[:, :R * R * C].reshape(K, R, R, C).float()
            if name == "stem":
                g = g[..., :zm.in_channels]
            out[name + ".weight"] = g.permute(0, 3, 1, 2)
            out[name + ".gamma"] = mod.gamma.grad.float()
            out[name + ".beta"] = mod.beta.grad.float()
    nc = zm.num_classes
    out["fc_w"] = zm.fc.weight.grad[:nc].float()
    out["fc_b"] = zm.fc.bias.grad[:nc].float()
    return out


def cos(a, b):
    return F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item()


def grad_report(zm, ref):
    zg = zoo_grad_views(zm)
    rp = dict(ref.named_parameters())
    rows = []
    for n, g in zg.items():
        r = rp[n].grad
        rel = ((g - r).norm() / r.norm().clamp_min(1e-30)).item()
        rows.append((n, cos(g, r), rel, r.norm().item()))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--warmup-steps", type=int, default=0)
    ap.add_argument("--repeat", action="store_true")
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--json", default="")
    ap.add_argument("--zero-gamma", action="store_true", help="zero-init the last BN gamma of every block")
    ap.add_argument("--nesterov", action="store_true")
    ap.add_argument("--base-lr", type=float, default=None, help="warmup start lr (default lr/warmup)")
    ap.add_argument("--autocast-ref", action="store_true", help="also report torch bf16-autocast grads vs fp32")
    a = ap.parse_args()

    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import resnet50
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine

    ctx = init_nncontext("parity")
    dev = ctx.device
    torch.manual_seed(1234)
    zm0 = resnet50(num_classes=1000, zero_init_residual=a.zero_gamma)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn(a.batch, 3, 224, 224, device=dev, generator=g)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)
    result = {}

    def lr_at(i):
        if a.warmup_steps and i < a.warmup_steps:
            b = a.base_lr if a.base_lr is not None else a.lr / a.warmup_steps
            return b + (a.lr - b) * i / a.warmup_steps
        return a.lr

    # ---- step-0 gradient parity ----
    ref = RefResNet(zm0).to(dev).train()
    if not a.no_ref:
        zm = copy.deepcopy(zm0).to(dev).train()
        for p in zm.parameters():
            p.grad = None
        lz = softmax_cross_entropy(zm(x), y)
        lz.backward()
        lr_ = F.cross_entropy(ref(x), y)
        lr_.backward()
        print("step0 loss native %.5f  fp32 %.5f" % (lz.item(), lr_.item()))
        rows = grad_report(zm, ref)
        print("%-34s %8s %8s %10s" % ("param", "cos", "relerr", "|g_ref|"))
        for n, c, rel, nr in rows:
            print("%-34s %8.5f %8.4f %10.3e" % (n, c, rel, nr))
        worst = sorted(rows, key=lambda r: r[1])[:5]
        print("worst cos:", [(n, round(c, 4)) for n, c, _, _ in worst])
        result["grad"] = [{"name": n, "cos": c, "rel": rel} for n, c, rel, _ in rows]
        if a.autocast_ref:
            # the same fp32 reference under torch bf16 autocast: how far does PyTorch's own bf16
            # path land from fp32 on this network (sensitivity of the gradient to rounding)
            g32 = {n: p.grad.clone() for n, p in ref.named_parameters()}
            ref2 = RefResNet(zm0).to(dev).train()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                l2 = F.cross_entropy(ref2(x).float(), y)
            l2.backward()
            print("%-34s %8s %8s | %8s" % ("param", "cos_ac", "rel_ac", "cos_zoo"))
            zc = {n: c for n, c, _, _ in rows}
            ac = []
            for n, p in ref2.named_parameters():
                c = cos(p.grad, g32[n])
                rel = ((p.grad - g32[n]).norm() / g32[n].norm().clamp_min(1e-30)).item()
                ac.append({"name": n, "cos": c, "rel": rel})
                print("%-34s %8.5f %8.4f | %8.5f" % (n, c, rel, zc[n]))
            result["grad_autocast"] = ac
            del ref2
        del zm
        ref.zero_grad(set_to_none=True)
        ref = RefResNet(zm0).to(dev).train()

    # ---- trajectories ----
    def run_native():
        zm = copy.deepcopy(zm0)
        opt = SGD(learningrate=a.lr, momentum=0.9, weightdecay=1e-4, dampening=0.0, nesterov=a.nesterov)
        eng = TrainingEngine(zm, softmax_cross_entropy, opt)
        losses = []
        for i in range(a.steps):
            opt.learning_rate = lr_at(i)
            losses.append(float(eng.train_step(x, y).float().item()))
        return losses

    def run_ref():
        opt = torch.optim.SGD(ref.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4, nesterov=a.nesterov)
        losses = []
        for i in range(a.steps):
            for pg in opt.param_groups:
                pg["lr"] = lr_at(i)
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(ref(x), y)
            loss.backward()
            opt.step()
            losses.append(loss.item())
        return losses

    ln = run_native()
    result["native"] = ln
    if a.repeat:
        result["native2"] = run_native()
    if not a.no_ref:
        result["fp32"] = run_ref()
    print("step  native    " + ("native2   " if a.repeat else "") + ("fp32" if not a.no_ref else ""))
    for i in range(a.steps):
        s = "%4d  %8.4f  " % (i, ln[i])
        if a.repeat:
            s += "%8.4f  " % result["native2"][i]
        if not a.no_ref:
            s += "%8.4f" % result["fp32"][i]
        print(s)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(result, f)


if __name__ == "__main__":
    main()
