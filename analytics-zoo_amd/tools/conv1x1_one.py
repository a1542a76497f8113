"""Run one 1x1 conv op N times (for rocprofv3 --pmc passes).  args: H Cin Cout op iters"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import zoo._C as C  # noqa: E402
from zoo.ops import _kern  # noqa: E402
H, Cin, Cout, op, iters = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
N = 256
dev = torch.device("cuda")
x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
w = (torch.randn(Cout, Cin, device=dev) / Cin ** 0.5).bfloat16()
dy = torch.randn(N, H, H, Cout, device=dev).bfloat16()
stats = torch.zeros(C.stat_len(Cout), device=dev)
for _ in range(iters):
    if op == "fwd":
        _kern.conv_fwd(x, w, 1, 1)
    elif op == "fwdstats":
        _kern.conv_fwd(x, w, 1, 1, stats=stats)
    else:
        _kern.conv_dgrad(dy, w, Cout, 1, 1, Cin, H, H)
torch.cuda.synchronize()
print("done")
