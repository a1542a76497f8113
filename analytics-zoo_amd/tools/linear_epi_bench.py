#!/usr/bin/env python3
"""Transformer-linear forward on the native GEMM with and without its epilogue work (bias,
activation) against hipBLASLt (F.linear) at the BERT-base b128 s128 shapes: isolates the cost of
the general epilogue (EPI 0) from the GEMM main loop. Interleaved rounds, median ms."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from zoo.ops import _kern  # noqa: E402
from zoo.ops.conv import bf16_weight  # noqa: E402
from tools.igemm2_bench import time_fns  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for (M, K, N) in [(16384, 768, 2304), (16384, 768, 768), (16384, 768, 3072), (16384, 3072, 768)]:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / math.sqrt(K))
        b = torch.randn(N, device=dev) * 0.1
        wb = bf16_weight(w)
        x4 = x.view(M, 1, 1, K)
        fns = {
            "lean": lambda: _kern.conv_fwd(x4, wb, 1, 1),
            "bias": lambda: _kern.conv_fwd(x4, wb, 1, 1, bias=b),
            "bias_relu": lambda: _kern.conv_fwd(x4, wb, 1, 1, bias=b, act=1),
            "bias_gelu": lambda: _kern.conv_fwd(x4, wb, 1, 1, bias=b, act=2),
            "hipblaslt_bias": lambda: F.linear(x, wb.view(N, K), b.bfloat16()),
        }
        ref = F.linear(x.float(), wb.view(N, K).float(), b)
        err = ((fns["bias"]().view(M, N).float() - ref).norm() / ref.norm()).item()
        ms = time_fns(fns)
        fl = 2.0 * M * N * K
        print(json.dumps({"gemm": [M, N, K], "err_bias": round(err, 5),
                          **{"us_" + k: round(v * 1e3, 1) for k, v in ms.items()},
                          **{"tf_" + k: round(fl / v / 1e9, 1) for k, v in ms.items()}}), flush=True)


if __name__ == "__main__":
    main()
