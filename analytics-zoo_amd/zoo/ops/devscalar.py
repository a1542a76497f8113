"""Per-step scalars that captured kernels read from device memory.

A hipGraph replays its kernels with the arguments of the capture: the learning rate, Adam's
bias corrections and the dropout seeds would freeze at their capture-step values. Kernels that
must follow the host's per-step values read them from a small device buffer instead
(``optim_device_hparams``, ``set_dropout_seed_offset`` in csrc/ops.cpp), and the host refreshes
that buffer before every step with one asynchronous host->device copy on the current stream --
ordered before the graph replay, never captured into it, and with no host synchronisation.
The host side of the copy is a small ring of pinned buffers; a slot is reused only once the
copy that last read it has completed (its event), so a later write cannot race an in-flight DMA.
"""
import torch


class DeviceStager:
    def __init__(self, n, dtype, device, ring=4):
        self.dev = torch.zeros(n, dtype=dtype, device=device)
        self._ring = [[torch.zeros(n, dtype=dtype).pin_memory(), None] for _ in range(ring)]
        self._i = 0

    def stage(self, values):
        slot = self._ring[self._i]
        if slot[1] is not None:
            slot[1].synchronize()
        slot[0].copy_(torch.tensor(values, dtype=slot[0].dtype))
        self.dev.copy_(slot[0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        slot[1] = ev
        self._i = (self._i + 1) % len(self._ring)
        return self.dev


_SEED = {}


def _key(device):
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


_USED = set()   # devices whose captured graphs contain dropout kernels that read the offset


def seed_offset_live(device):
    """Whether the dropout kernels of ``device`` read a per-step device seed offset. Called by the
    dropout paths while a graph is being captured; a True answer there also records that the
    graph needs the offset restaged before its replays (``seed_offset_used``)."""
    k = _key(device)
    live = k in _SEED
    if live and torch.cuda.is_current_stream_capturing():
        _USED.add(k)
    return live


def seed_offset_used(device):
    """Whether any graph captured on ``device`` reads the dropout seed offset."""
    return _key(device) in _USED


def dropout_seed_stager(device):
    """The process-wide dropout seed offset of ``device`` (created and registered with the
    kernels on first use; never freed, since every later dropout launch reads it)."""
    key = _key(device)
    st = _SEED.get(key)
    if st is None:
        from zoo.ops._native import native
        st = DeviceStager(1, torch.int32, device)
        native().set_dropout_seed_offset(st.dev)
        _SEED[key] = st
    return st
