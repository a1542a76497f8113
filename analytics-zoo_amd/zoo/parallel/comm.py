"""Native communicator: the C++ comm layer (csrc/comm.cpp) over RCCL, bootstrapped through an
existing torch.distributed group.

``NativeComm(group)`` creates one RCCL communicator for the ranks of ``group``: rank 0 of the
group draws the unique id, ``torch.distributed.broadcast_object_list`` hands it to the others
(over the group's own backend), every rank calls ``comm_init``. Collectives are enqueued on the
CURRENT HIP stream -- GradSync issues them inside its comm-stream context, so they order against
the backward exactly like the ProcessGroup path, without its per-call work objects. The channel
count comes from ``ZooConfig.rccl_channels`` (0: RCCL's default).

Reference parity: BigDL AllReduceParameter / §5.8's C++ comm layer.
"""
import torch
import torch.distributed as dist

from zoo.ops._native import native


class NativeComm:
    def __init__(self, group=None, channels=0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        m = native()
        uid = [m.comm_unique_id() if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(uid, src=src, group=group)
        self.h = m.comm_init(uid[0], self.world, self.rank, int(channels))
        self._m = m

    # the ProcessGroup-shaped calls GradSync uses --------------------------------------------
    def all_reduce(self, t, op="sum"):
        self._m.comm_all_reduce(self.h, t, op)

    def reduce_scatter(self, out, inp, op="sum"):
        self._m.comm_reduce_scatter(self.h, out, inp, op)

    def all_gather(self, out, inp):
        self._m.comm_all_gather(self.h, out, inp)

    def all_to_all(self, out, inp):
        self._m.comm_all_to_all(self.h, out, inp)

    def broadcast(self, t, root=0):
        self._m.comm_broadcast(self.h, t, root)

    def fused(self):
        """``with comm.fused():`` fuses the enclosed collectives into one RCCL launch group."""
        return _Group(self._m)

    def close(self):
        if self.h is not None:
            self._m.comm_destroy(self.h)
            self.h = None


class _Group:
    def __init__(self, m):
        self._m = m

    def __enter__(self):
        self._m.comm_group_start()
        return self

    def __exit__(self, *exc):
        self._m.comm_group_end()
        return False


def native_comm_ok(group=None):
    """The native layer needs GPU tensors and an RCCL-backed group."""
    return (dist.is_available() and dist.is_initialized() and torch.cuda.is_available()
            and dist.get_backend(group) == "nccl")
