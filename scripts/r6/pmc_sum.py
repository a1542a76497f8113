#!/usr/bin/env python3
"""Sum a rocprofv3 counter_collection CSV per (kernel, counter): mean per dispatch."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(float)
cnt = defaultdict(int)
for path in sys.argv[1:]:
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r.get("Kernel_Name", "")[:60]
            c = r.get("Counter_Name", "")
            acc[(k, c)] += float(r.get("Counter_Value", 0) or 0)
            cnt[(k, c)] += 1
keys = sorted({k for k, _ in acc})
for k in keys:
    if "convlstm" not in k and "wgrad" not in k:
        continue
    items = ["%s=%.4g" % (c, acc[(k2, c)] / max(1, cnt[(k2, c)])) for (k2, c) in sorted(acc) if k2 == k]
    print(k, " | ".join(items))
