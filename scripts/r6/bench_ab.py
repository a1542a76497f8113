#!/usr/bin/env python3
"""bench.py with one module-level switch set first: bench_ab.py MODULE ATTR VALUE [bench args]"""
import os
import runpy
import sys

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(root, "analytics-zoo_amd"))
import importlib  # noqa: E402

mod, attr, val = sys.argv[1:4]
setattr(importlib.import_module(mod), attr, {"True": True, "False": False}.get(val, val))
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[4:]
runpy.run_path(sys.argv[0], run_name="__main__")
