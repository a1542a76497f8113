"""Weight-gradient side stream.

In a backward pass the critical path is the data-gradient chain (BN backward -> dgrad -> the
previous layer's BN backward ...); the weight gradients hang off it and nothing in the same
backward reads them. Inside the training engine's backward (``enabled(dev)``) the native
conv / linear backwards issue their weight-gradient launches (wgrad + split-K fold) on one
side stream per device: the side stream first waits for everything the compute stream has
issued so far (x and dy are ready), the launches then overlap the following dgrad / BN
kernels -- filling the tail of each persistent kernel and the launch gaps -- and ``join`` (end
of backward, before any reader of the gradients) makes the compute stream wait for them.
Tensors the side launches read are ``record_stream``-ed, so the caching allocator does not
hand their memory to the compute stream early. Under hipGraph capture the fork / join are
captured as graph edges.

Outside an ``enabled`` scope (user code calling ``loss.backward()`` then reading ``.grad``)
everything stays on the current stream. ``ZOO_WGRAD_STREAM=0`` turns the side stream off.
Reference parity: BigDL's DistriOptimizer overlaps parameter-gradient work with the backward
of the remaining layers per model replica; this is the single-GPU form.
"""
import contextlib
import os

import torch

_ON = os.environ.get("ZOO_WGRAD_STREAM", "1") != "0"
_side = {}        # device index -> torch.cuda.Stream
_enabled = set()  # device indices inside an engine backward
_used = set()     # device indices with side work not yet joined


def on():
    return _ON


def _stream(idx):
    s = _side.get(idx)
    if s is None:
        # the whole device: a CU-masked side stream (16-64 CUs) ran the ResNet-50 step 28-32 %
        # slower (profiles/r5/ab_side_cus_r5.md)
        s = torch.cuda.Stream(device=idx)
        _side[idx] = s
    return s


@contextlib.contextmanager
def enabled(dev):
    """Engine scope: weight gradients of this backward may run on the side stream."""
    if not _ON or dev.type != "cuda":
        yield
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    _stream(idx)
    _enabled.add(idx)
    try:
        yield
    finally:
        _enabled.discard(idx)
        join(dev)


def active(dev):
    return dev.type == "cuda" and (dev.index if dev.index is not None else torch.cuda.current_device()) in _enabled


@contextlib.contextmanager
def wgrad(dev, *reads, on=True):
    """Run the enclosed weight-gradient launches (and their gradient-ready notifications) on
    the side stream when the engine enabled it; ``reads`` are the tensors they read. ``on``:
    False when the gradient is returned to autograd (consumed on the compute stream)."""
    if not on or not active(dev):
        yield
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _side[idx]
    s.wait_stream(torch.cuda.current_stream(idx))
    with torch.cuda.stream(s):
        yield
    for t in reads:
        if t is not None and t.is_cuda:
            t.record_stream(s)
    _used.add(idx)


def side_for(dev):
    """The side stream of ``dev`` (created on first use)."""
    return _stream(dev.index if dev.index is not None else torch.cuda.current_device())


def mark_used(dev):
    """Work was issued on the side stream outside ``wgrad`` (the in-backward optimizer)."""
    _used.add(dev.index if dev.index is not None else torch.cuda.current_device())


def pending(dev):
    """The side stream of ``dev`` if it has unjoined work (collectives must wait for it too)."""
    if dev.type != "cuda":
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    return _side[idx] if idx in _used else None


def join(dev):
    """Make the current stream of ``dev`` wait for its side-stream weight gradients."""
    if dev.type != "cuda":
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx in _used:
        torch.cuda.current_stream(idx).wait_stream(_side[idx])
        _used.discard(idx)
