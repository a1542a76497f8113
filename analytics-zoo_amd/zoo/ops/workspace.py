"""Per-step zeroed scratch for small fp32 accumulators (BN statistics / sums).

Every conv+BN unit needs 2*C zero-initialised fp32 accumulators in forward and
again in backward. Allocating each with ``torch.zeros`` costs one fill launch
apiece (~100 launches per ResNet-50 step); instead the engine zeroes ONE
buffer at the start of each step (a single memset) and ops bump-allocate from
it. Outside an engine step (or when the buffer is exhausted) ops fall back to
``torch.zeros``; the high-water mark grows the buffer for the next step.

The memset covers the high-water mark of EVERY step run so far -- eager steps and
hipGraph captures alike. A captured step replays its own kernels (and its own memset,
sized when it was captured) without running this module, so an eager step after replays
of a larger graph still finds every slot those replays dirtied cleared. A buffer that is
replaced by a larger one is kept alive: captured graphs keep reading and writing it.
"""
import torch

_state = {"buf": None, "off": 0, "active": False, "need": 1 << 16, "hw": 0, "retired": []}


def begin_step(device):
    buf = _state["buf"]
    need = _state["need"]
    if buf is None or buf.device != torch.device(device) or buf.numel() < need:
        if buf is not None:
            _state["retired"].append(buf)   # graphs captured over it still use it
        _state["buf"] = torch.zeros(max(need, 1 << 16), dtype=torch.float32, device=device)
        _state["hw"] = 0
    elif _state["hw"] > 0:
        buf[:_state["hw"]].zero_()   # every slot any step (or captured graph) handed out
    _state["off"] = 0
    _state["active"] = True


def end_step():
    _state["active"] = False
    _state["hw"] = max(_state["hw"], _state["off"])


def high_water():
    """Elements of the current buffer that some step has used (zeroed by every begin_step)."""
    return _state["hw"]


def zeros(n, device):
    n = int(n)
    buf = _state["buf"]
    if _state["active"] and buf is not None and buf.device == torch.device(device):
        off = (_state["off"] + 63) // 64 * 64
        if off + n <= buf.numel():
            _state["off"] = off + n
            return buf[off:off + n]
        _state["need"] = max(_state["need"], 2 * (off + n))
    return torch.zeros(n, dtype=torch.float32, device=device)
