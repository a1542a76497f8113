"""Debug: is the ResNet-50 forward deterministic at small shapes? Two forwards of the same
model on the same input; report per-module output differences (first differing module)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "analytics-zoo_amd"))
import torch
from zoo.common.nncontext import init_nncontext
from zoo.models.image.resnet import resnet50
init_nncontext("dbg")
gpu = torch.device("cuda")
for (B, HW) in ((16, 64), (16, 224), (64, 64)):
    torch.manual_seed(0)
    m = resnet50(num_classes=10).to(gpu)
    x = torch.randn(B, 3, HW, HW, device=gpu)
    for mode in ("train", "eval"):
        getattr(m, mode)()
        outs = []
        for rep in range(3):
            rec = []
            hs = [mod.register_forward_hook(lambda mod, i, o, rec=rec, n=n: rec.append((n, o.detach().float().clone() if torch.is_tensor(o) else None)))
                  for n, mod in m.named_modules() if n]
            with torch.no_grad():
                m(x)
            for h in hs:
                h.remove()
            outs.append(rec)
        first = None
        worst = 0.0
        for (n, a), (_, b) in zip(outs[0], outs[1]):
            if a is None or b is None or a.shape != b.shape:
                continue
            d = ((a - b).abs().max() / a.abs().max().clamp_min(1e-6)).item()
            worst = max(worst, d)
            if d > 1e-2 and first is None:
                first = (n, tuple(a.shape), d)
        print(B, HW, mode, "worst rel diff", round(worst, 5), "first >1e-2:", first, flush=True)
