"""Multi-process JPEG decode for the serving worker.

PIL (libjpeg-turbo) holds the GIL for most of a decode, so a thread pool in the
worker process tops out at ~4k 256x256 images/s however many cores the box has
(``profiles/serving_r2.md``). The reference decodes in Spark executor threads on
the JVM (``Zs/serving/ClusterServing.scala:192-203`` PreProcessing), which has no
such lock. Here the decode runs in a pool of spawned helper processes (numpy +
PIL only, they never touch the GPU) that write RGB pixels straight into a ring of
shared-memory batch slots; the worker pins each slot with ``hipHostRegister`` once,
so a decoded batch goes to HBM with a single async copy.
"""
import multiprocessing as mp
import os
import sys

import numpy as np

# The helpers run the functions of ``_zoo_decode_worker.py`` (this directory), imported as
# a TOP-LEVEL module so that a spawned helper unpickles them without importing the ``zoo``
# package (and torch): helpers start in well under a second and hold no GPU state.
_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.append(_HERE)
import _zoo_decode_worker as _w  # noqa: E402


class ProcDecodePool:
    """``decode(payloads) -> pinned uint8 torch tensor [B, H, W, 3]`` (RGB) or None when
    the images do not all share one size (the caller then takes the generic path)."""

    def __init__(self, nproc=None, nslots=5):
        self.nproc = int(nproc or os.environ.get("ZOO_SERVING_DECODE_PROCS", "8"))
        self.nslots = nslots
        self.pool = mp.get_context("spawn").Pool(self.nproc)
        self.rings = {}   # (B, H, W) -> (shm, ndarray, [pinned tensors], next slot)

    def _ring(self, B, h, w):
        key = (B, h, w)
        r = self.rings.get(key)
        if r is None:
            import torch
            from multiprocessing import shared_memory
            shape = (self.nslots, B, h, w, 3)
            shm = shared_memory.SharedMemory(create=True, size=int(np.prod(shape)))
            arr = np.ndarray(shape, np.uint8, buffer=shm.buf)
            views = [torch.from_numpy(arr[s]) for s in range(self.nslots)]
            if torch.cuda.is_available():
                cudart = torch.cuda.cudart()
                # page-lock the shared block so H2D copies of a slot are async DMA
                cudart.cudaHostRegister(arr.ctypes.data, arr.nbytes, 0)
            r = self.rings[key] = [shm, arr, views, 0, shape]
        return r

    def decode(self, payloads):
        if not payloads:
            return None
        w, h = _w.probe_size(payloads[0])
        B = len(payloads)
        r = self._ring(B, h, w)
        slot = r[3] % self.nslots
        r[3] += 1
        step = (B + self.nproc - 1) // self.nproc
        tasks = [(r[0].name, r[4], slot, o, payloads[o:o + step]) for o in range(0, B, step)]
        if not all(self.pool.starmap(_w.decode_into, tasks)):
            return None
        return r[2][slot]

    def close(self):
        import torch
        self.pool.terminate()
        for r in self.rings.values():
            shm, arr = r[0], r[1]
            if torch.cuda.is_available():
                try:
                    torch.cuda.cudart().cudaHostUnregister(arr.ctypes.data)
                except Exception:  # noqa: BLE001
                    pass
            r[1] = r[2] = None
            del arr
            try:
                shm.close()
            except BufferError:   # a caller still holds a slot tensor: unlink only
                pass
            shm.unlink()
        self.rings.clear()
