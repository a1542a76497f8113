"""Py/xshard/shard.py names: DataShards / RayDataShards / RayPartition over the
thread/process-pool XShards of this package (no Ray actors: one process per GPU
takes its share with ``partition_by_rank``)."""
from zoo.xshard import XShards

DataShards = XShards
RayDataShards = XShards


class RayPartition:
    """A partition's list of shards (Py/xshard/shard.py:91-100)."""

    def __init__(self, shard_list):
        self.shard_list = shard_list

    def get_data(self):
        return [s.get_data() if hasattr(s, "get_data") else s for s in self.shard_list]
