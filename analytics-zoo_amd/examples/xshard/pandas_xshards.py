#!/usr/bin/env python3
"""XShards of pandas DataFrames (pyzoo/zoo/examples/xshard/ray-pandas.py): read a directory
of CSVs into shards, transform every shard in parallel, repartition and collect."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--csv-dir", default=None)
    ap.add_argument("--files", type=int, default=4)
    a = ap.parse_args(argv)
    import pandas as pd
    from zoo import xshard
    tmp = None
    d = a.csv_dir
    if d is None:
        tmp = tempfile.TemporaryDirectory()
        d = tmp.name
        rng = np.random.default_rng(0)
        for i in range(a.files):
            pd.DataFrame({"user": rng.integers(0, 100, 50), "value": rng.random(50)}).to_csv(
                os.path.join(d, "part%d.csv" % i), index=False)
    shards = xshard.read_csv(d)
    print("partitions:", shards.num_partitions())
    scaled = shards.apply(lambda df, k: df.assign(value=df["value"] * k), 10.0)
    two = scaled.repartition(2)
    total = two.concat()
    print("rows:", len(total), "mean value:", float(total["value"].mean()))
    if tmp is not None:
        tmp.cleanup()
    return len(total)


if __name__ == "__main__":
    main()
