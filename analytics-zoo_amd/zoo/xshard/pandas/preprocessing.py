"""Py/xshard/pandas/preprocessing.py names (read_csv / read_json / read_file_ray,
RayPandasShard) on top of the pooled XShards reader."""
from zoo.xshard import XShards, read_csv, read_json  # noqa: F401


def read_file_ray(context, file_path, file_type):
    return {"csv": read_csv, "json": read_json}[file_type](file_path, context)


class RayPandasShard:
    """One pandas partition (the reference's Ray actor state)."""

    def __init__(self, data=None):
        self.data = data

    def read_file_partitions(self, paths, file_type):
        import pandas as pd
        reader = pd.read_csv if file_type == "csv" else pd.read_json
        self.data = pd.concat([reader(p) for p in paths], ignore_index=True)

    def apply(self, func, *args):
        self.data = func(self.data, *args)
        return 0

    def get_data(self):
        return self.data
