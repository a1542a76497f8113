#!/usr/bin/env python3
"""Per-segment cycle shares of the persistent 3x3 kernel (c3.hip) from its diagnostic stamp
build: run with ZOO_C3_STAMPS=1.   python c3_stamps.py [--batch 256] [--dgrad]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import zoo._C as C  # noqa: E402
from zoo.ops import _kern  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dgrad", action="store_true")
    a = ap.parse_args()
    assert os.environ.get("ZOO_C3_STAMPS"), "set ZOO_C3_STAMPS=1"
    dev = torch.device("cuda")
    x = torch.randn(a.batch, 56, 56, 64, device=dev).bfloat16()
    w = (torch.randn(64, 576, device=dev) / math.sqrt(576)).bfloat16()
    stats = torch.zeros(128, device=dev)
    for _ in range(3):
        if a.dgrad:
            _kern.conv_dgrad(x, w, 64, 3, 3, 64, 56, 56, (1, 1), (1, 1))
        else:
            _kern.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=stats)
    torch.cuda.synchronize()
    v = np.array(C.c3_stamps(), dtype=np.float64).reshape(-1, 4, 5)
    bands = v[:, :, 4].sum()
    names = ["row prefetch + operand issue", "MFMA taps", "epilogue", "wait + barrier"]
    tot = v[:, :, :4].sum()
    print("workgroups %d, band-waves %d, cycles per band per wave %.0f" % (v.shape[0], bands, tot / bands))
    for k, n in enumerate(names):
        s = v[:, :, k].sum()
        print("  %-30s %6.1f%%  %8.0f cyc/band" % (n, 100 * s / tot, s / bands))


if __name__ == "__main__":
    main()
