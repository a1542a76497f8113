#!/usr/bin/env python3
"""Full names of the non-zoo (PyTorch / runtime) dispatches of the last complete step in a
rocprofv3 kernel-trace database (the step marker as in prof_step.py)."""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "analytics-zoo_amd", "tools"))
from prof_step import load_rows, pick_step  # noqa: E402

rows = load_rows(sys.argv[1])
step = pick_step(rows, re.compile(sys.argv[2] if len(sys.argv) > 2 else r"nchw_to_s2d_kernel|nhwc_u8_to_s2d"), 1)
for i, r in enumerate(step):
    if "zoo::" in r["name"]:
        continue
    print("%3d %7.1f us  %s" % (i, r["dur"] / 1e3, r["name"][:400]))
