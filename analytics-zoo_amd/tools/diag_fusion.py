"""Run-to-run / fused-vs-unfused gradient agreement of a small ResNet on the GPU."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import zoo.models.image.resnet as R  # noqa: E402
from zoo.ops import softmax_cross_entropy  # noqa: E402


def run(m, x, y, fuse):
    R.FUSE_BN_BACKWARD = fuse
    m.zero_grad(set_to_none=True)
    out = m(x)
    loss = softmax_cross_entropy(out, y)
    loss.backward()
    return out.detach().float().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}


def cmp(tag, a, b):
    worst = []
    for n in a:
        u, v = a[n].flatten().double(), b[n].flatten().double()
        c = F.cosine_similarity(u, v, dim=0).item()
        worst.append((c, n, ((u - v).norm() / u.norm().clamp_min(1e-30)).item()))
    worst.sort()
    print(tag, "worst", [(n, round(c, 5), round(r, 4)) for c, n, r in worst[:6]],
          "best", [(n, round(c, 5)) for c, n, _ in worst[-3:]])


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    blk = R.Bottleneck if (len(sys.argv) < 2 or sys.argv[1] == "bottleneck") else R.BasicBlock
    m = R.ResNet(blk, [2, 2, 1, 1], num_classes=16, width=16).to(dev)
    x = torch.randn(8, 3, 96, 96, device=dev)
    y = torch.randint(0, 16, (8,), device=dev)
    o1, g1 = run(m, x, y, False)
    o2, g2 = run(m, x, y, False)
    o3, g3 = run(m, x, y, True)
    o4, g4 = run(m, x, y, True)
    print("fwd diff u/u", (o1 - o2).abs().max().item(), "u/f", (o1 - o3).abs().max().item())
    cmp("unfused-vs-unfused", g1, g2)
    cmp("unfused-vs-fused", g1, g3)
    cmp("fused-vs-fused", g3, g4)
    m.eval()
    with torch.no_grad():
        e1 = m(x).float()
        e2 = m(x).float()
    print("eval diff", (e1 - e2).abs().max().item())


if __name__ == "__main__":
    main()
