"""Shared bits of the examples: sys.path setup and the device argument."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def add_common(ap):
    ap.add_argument("--seed", type=int, default=0)
    return ap
