"""ResNet-50 inference throughput: bf16 (fused conv+BN kernels) vs int8 (zoo.ops.quant).
python tools/quant_bench.py [--batch 64] [--iters 20]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from zoo.models.image.resnet import resnet50  # noqa: E402
from zoo.ops import quant as Q  # noqa: E402


def bench(m, x, iters):
    with torch.no_grad():
        for _ in range(3):
            m(x)
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(iters):
            m(x)
        torch.cuda.synchronize()
    return (time.time() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    m = resnet50().cuda().eval()
    x = torch.randn(a.batch, 3, 224, 224, device="cuda")
    tb = bench(m, x, a.iters)
    Q.quantize(m)
    tq = bench(m, x, a.iters)
    print("resnet50 inference batch %d: bf16 %.2f ms (%.0f img/s) | int8 %.2f ms (%.0f img/s)"
          % (a.batch, tb * 1e3, a.batch / tb, tq * 1e3, a.batch / tq), flush=True)


if __name__ == "__main__":
    main()
