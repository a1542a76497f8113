"""Decode helpers run inside the spawned processes of zoo/serving/decode_pool.py
(numpy + PIL only; imported there as a top-level module, see decode_pool.py)."""
import numpy as np

_ATTACHED = {}


def attach(name, shape):
    from multiprocessing import shared_memory
    a = _ATTACHED.get(name)
    if a is None:
        # (spawned helpers share the worker's resource tracker: attaching re-registers the
        # same name, a no-op, and the worker unlinks the block in ProcDecodePool.close)
        shm = shared_memory.SharedMemory(name=name)
        a = _ATTACHED[name] = (shm, np.ndarray(shape, np.uint8, buffer=shm.buf))
    return a[1]


def decode_into(name, shape, slot, offset, payloads):
    """Decode JPEG/PNG payloads into ring[slot, offset + i]; returns False on a size mismatch."""
    import io
    from PIL import Image
    ring = attach(name, shape)
    h, w = shape[2], shape[3]
    for i, p in enumerate(payloads):
        im = Image.open(io.BytesIO(p))
        im.draft("RGB", None)
        if im.mode != "RGB":
            im = im.convert("RGB")
        if im.size != (w, h):
            return False
        ring[slot, offset + i] = np.asarray(im)
    return True


def probe_size(payload):
    import io
    from PIL import Image
    with Image.open(io.BytesIO(payload)) as im:
        return im.size
