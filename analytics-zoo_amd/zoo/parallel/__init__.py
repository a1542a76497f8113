"""Parallelism: flat parameter store, RCCL gradient sync (all-reduce / ZeRO-1 sharded)."""
from zoo.parallel.flat import FlatParams
from zoo.parallel.ddp import GradSync, global_norm_clip, constant_clip
