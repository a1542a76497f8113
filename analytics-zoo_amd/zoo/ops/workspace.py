"""Per-step zeroed scratch for small fp32 accumulators (BN statistics / sums).

Every conv+BN unit needs 2*C zero-initialised fp32 accumulators in forward and
again in backward. Allocating each with ``torch.zeros`` costs one fill launch
apiece (~100 launches per ResNet-50 step); instead the engine zeroes ONE
buffer at the start of each step (a single memset) and ops bump-allocate from
it. Outside an engine step (or when the buffer is exhausted) ops fall back to
``torch.zeros``; the high-water mark grows the buffer for the next step.
"""
import torch

_state = {"buf": None, "off": 0, "active": False, "need": 1 << 16}


def begin_step(device):
    buf = _state["buf"]
    need = _state["need"]
    if buf is None or buf.device != torch.device(device) or buf.numel() < need:
        _state["buf"] = torch.zeros(max(need, 1 << 16), dtype=torch.float32, device=device)
    elif _state["off"] > 0:
        buf[:_state["off"]].zero_()   # only what the last step handed out is dirty (none: no launch)
    _state["off"] = 0
    _state["active"] = True


def end_step():
    _state["active"] = False


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
