"""XShards: partitioned pandas data (Py/xshard/shard.py:20-100, xshard/pandas/preprocessing.py:26-189).

The reference distributes pandas partitions over Ray actors. Here a shard
set is a list of DataFrames; ``apply`` runs the function on every partition
with a thread / process pool, ``read_csv`` / ``read_json`` split input files
(or one large file, by rows) into partitions, and ``partition_by_rank``
gives each GPU process its share for one-process-per-GPU training.
"""
import glob
import os
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor

import numpy as np
import pandas as pd


class XShards:
    def __init__(self, partitions, num_workers=None, use_processes=False):
        self.partitions = list(partitions)
        self.num_workers = num_workers or min(8, max(1, len(self.partitions)))
        self.use_processes = use_processes

    def _pool(self):
        return (ProcessPoolExecutor if self.use_processes else ThreadPoolExecutor)(self.num_workers)

    def apply(self, func, *args):
        with self._pool() as ex:
            parts = list(ex.map(lambda p: func(p, *args), self.partitions)) if not self.use_processes else \
                list(ex.map(func, self.partitions, *[[a] * len(self.partitions) for a in args]))
        return XShards(parts, self.num_workers, self.use_processes)

    transform_shard = apply

    def collect(self):
        return list(self.partitions)

    def num_partitions(self):
        return len(self.partitions)

    def get_partitions(self):
        return self.partitions

    def repartition(self, num_partitions):
        df = pd.concat(self.partitions, ignore_index=True) if self.partitions else pd.DataFrame()
        bounds = np.linspace(0, len(df), num_partitions + 1).astype(int)
        parts = [df.iloc[bounds[i]:bounds[i + 1]].reset_index(drop=True) for i in range(num_partitions)]
        return XShards(parts, self.num_workers, self.use_processes)

    def partition_by_rank(self):
        from zoo.common.nncontext import get_nncontext
        ctx = get_nncontext()
        return XShards(self.partitions[ctx.rank::ctx.world_size], self.num_workers, self.use_processes)

    def concat(self):
        return pd.concat(self.partitions, ignore_index=True)


def _files(path, ext):
    if os.path.isdir(path):
        return sorted(glob.glob(os.path.join(path, "*" + ext))) or sorted(glob.glob(os.path.join(path, "*")))
    return sorted(glob.glob(path))


def _read(path, reader, num_partitions, ext="", **kwargs):
    files = _files(path, ext)
    if not files:
        raise FileNotFoundError(path)
    with ThreadPoolExecutor(min(8, len(files))) as ex:
        dfs = list(ex.map(lambda f: reader(f, **kwargs), files))
    if num_partitions is None or num_partitions == len(dfs):
        return XShards(dfs)
    return XShards(dfs).repartition(num_partitions)


def read_csv(file_path, context=None, num_partitions=None, **kwargs):
    return _read(file_path, pd.read_csv, num_partitions, ".csv", **kwargs)


def read_json(file_path, context=None, num_partitions=None, **kwargs):
    return _read(file_path, pd.read_json, num_partitions, ".json", **kwargs)
