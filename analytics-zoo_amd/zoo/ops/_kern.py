"""Thin keyword wrappers over the raw ``zoo._C`` conv entry points, plus the
convolution data-gradient driver.

``conv_dgrad`` computes dX of an NHWC conv:
  * stride 1: ONE transposed-conv launch (flipped filter, pad R-1-p).
  * stride s > 1: the transposed conv would waste (s^2-1)/s^2 of the MFMA work
    on zero-inserted rows, so the output is split into its s_h x s_w parity
    classes; each class is a stride-1 conv of dY with a flipped SUB-filter
    (the taps r = r0 + s*t that reach that class), written straight to its
    strided output positions by the igemm epilogue's row remap. Classes no
    tap reaches are zero.
"""
import math

import os

import torch

from zoo.ops._native import native


def conv_fwd(x, w, R, S, stride=(1, 1), pad=(0, 0), dil=(1, 1), ldil=(1, 1), bias=None, resid=None, stats=None,
             act=0, out_f32=False, out_bf16=True, out_hw=(0, 0), out=None, omap=None, bstats=None, pro=None,
             resid_half=False, pro_fwd=None, act_pre=None):
    """``bstats = (z or None, y, mean, inv, sums[, gamma, beta[, y2, sums2]])`` fuses the producing unit's
    BN-backward reduction (and ReLU mask) into this conv's epilogue. The mask source: a bf16
    ``z`` (ReLU output), a uint8 ``z`` (1-bit mask of the forward apply), or -- z None and
    gamma given -- recomputed from ``y`` with the unit's affine (csrc/kernels/bnmask.h).
    ``pro = (y, coef, dy_out or None)``: ``x`` is a unit's masked output gradient g and the GEMM
    runs on that unit's BN backward dy = A g + B y + Cc instead (the BN-backward prologue,
    csrc/kernels/bnfold.hip); dy is written to ``dy_out``.
    ``resid_half``: ``resid`` is [N, P/2, Q/2, K], added at the even output positions only (the
    compact data gradient of a 1x1 stride-2 shortcut, :func:`conv_dgrad_s2_compact`).
    ``pro_fwd = (coef, z_out)``: ``x`` is a conv -> BN -> ReLU unit's pre-BN output y and the GEMM
    runs on that unit's z = relu(coef[c] y + coef[2C + c]), which is also written to ``z_out`` (the
    forward consumer-side apply; ``coef`` from ``bn_fwd_coef``). ``pro_fwd = (coef, z_out, resid, rcoef,
    mask)``: the unit has a residual -- z = relu(A y + Cc + R), R = resid or rA resid + rC (rcoef, a
    projection shortcut's BatchNorm) -- and its 1-bit ReLU mask goes to ``mask`` (pw.hip EPI 4).
    ``act_pre`` (GELU only): the pre-activation is also written there (bf16, the output's shape)
    -- from the large-tile kernel's epilogue, or by a separate GELU pass for other shapes."""
    bz = by = bm = bi = bsum = bg = bb = by2 = bsum2 = None
    if bstats is not None:
        bz, by, bm, bi, bsum = bstats[:5]
        if len(bstats) > 5:
            bg, bb = bstats[5], bstats[6]
        if len(bstats) > 7:
            by2, bsum2 = bstats[7], bstats[8]
    py, pc, pd = pro if pro is not None else (None, None, None)
    prc = pmask = None
    if pro_fwd is not None:
        pc, pd = pro_fwd[0], pro_fwd[1]
        if len(pro_fwd) > 2:
            py, prc, pmask = pro_fwd[2], pro_fwd[3], pro_fwd[4]
    return native().conv_fwd(x, w, R, S, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], ldil[0], ldil[1],
                             bias, resid, stats, act, out_f32, out_bf16, out_hw[0], out_hw[1], out,
                             list(omap) if omap else [], bz, by, bm, bi, bsum, bg, bb, py, pc, pd, bool(resid_half),
                             pro_fwd is not None, prc, pmask, act_pre, by2, bsum2)


# ---------------------------------------------------------------------------
# Flipped dgrad filters, refreshed in ONE batched launch per weight update.
#
# Every dgrad needs its filter flipped to [Cin][R][S][Cout] (and strided convs one
# sub-filter per output-parity class). Done per call that is one small launch per conv
# per backward (62 on ResNet-50, profiles/resnet50_b256_r2_lean.md). For weights that
# live in a FlatParams bf16 buffer -- rewritten only by the fused optimizer kernels and
# refresh_bf16, which bump ``weights_epoch`` -- the flipped copies are cached, and the
# first dgrad after an update re-flips ALL cached filters with one
# ``flip_weights_batched`` launch. Other weights (inference, plain modules) and calls
# made while a hipGraph is being captured flip directly, as before.
# ---------------------------------------------------------------------------
_EPOCH = [0]
_CACHE_ON = True
_FLATS = {}             # id(FlatParams.bf16) -> weakref(FlatParams)


def bump_weights_epoch():
    """Called by every writer of a FlatParams bf16 buffer (optimizer steps, refresh_bf16)."""
    _EPOCH[0] += 1


def weights_epoch():
    return _EPOCH[0]


_STATS_EPOCH = [0]


def bump_stats_epoch():
    """Called whenever a native training-mode BatchNorm forward rewrites running statistics
    through raw pointers (no ``_version`` bump): caches derived from running stats (the
    eval-mode BN fold) key on this."""
    _STATS_EPOCH[0] += 1


def stats_epoch():
    return _STATS_EPOCH[0]


def register_flat(flat):
    """Give a FlatParams its own flip cache (it dies with the FlatParams, so cached
    pointers never outlive the buffer they point into)."""
    import weakref
    if flat.bf16 is not None and flat.bf16.is_cuda:
        for k in [k for k, r in _FLATS.items() if r() is None]:
            del _FLATS[k]
        _FLATS[id(flat.bf16)] = weakref.ref(flat)
        flat._flip_cache = _FlipCache()
        bump_weights_epoch()


def _owner_cache(w):
    """The flip cache of the FlatParams whose bf16 buffer ``w`` is a view of, else None."""
    if not _CACHE_ON or not _FLATS or not w.is_cuda:
        return None
    base = w._base if w._base is not None else w
    ref = _FLATS.get(id(base))
    f = ref() if ref is not None else None
    if f is None or f.bf16 is not base:
        return None
    return getattr(f, "_flip_cache", None)


class _FlipCache:
    def __init__(self):
        self.entries = {}     # key -> [w, wt, epoch]
        self.table = None     # device int32 [n, desc_ints]
        self.table_n = 0
        self.nblocks = 0
        self.pending = None   # event of a prefetched re-flip on the side stream (prefetch)
        self.cap_gen = -1     # the capture whose graph already holds a batched re-flip

    def prefetch(self, side):
        """Re-flip every cached filter now, on ``side``, if the weights changed since the last
        flip: issued at the start of a training step, the batched flip overlaps the forward
        instead of sitting on the data-gradient chain in front of the first dgrad."""
        ep = _EPOCH[0]
        if not self.entries or all(e[2] == ep for e in self.entries.values()):
            return
        if self.table is None or self.table_n != len(self.entries):
            self._build_table()
        dev = self.table.device
        side.wait_stream(torch.cuda.current_stream(dev))   # the last update of the weights
        with torch.cuda.stream(side):
            native().flip_weights_batched(self.table, self.table_n, self.nblocks)
            ev = torch.cuda.Event()
            ev.record(side)
        for e in self.entries.values():
            e[2] = ep
        self.pending = ev

    def _build_table(self):
        import numpy as np
        m = native()
        di = m.flip_desc_ints()
        ents = list(self.entries.items())
        arr = np.zeros((len(ents), di), dtype=np.int32)
        ptrs = arr[:, 0:4].copy().view(np.int64)
        blk = 0
        for i, (key, (w, wt, _)) in enumerate(ents):
            _, K, R, S, C, r0, s0, Ra, Sb, sh, sw = key
            total = C * Ra * Sb * K
            nblk = max(1, min(256, (total + 1023) // 1024))
            ptrs[i, 0] = w.data_ptr()
            ptrs[i, 1] = wt.data_ptr()
            arr[i, 4:18] = (K, R, S, C, w.shape[1], r0, s0, Ra, Sb, sh, sw, wt.shape[1], blk, nblk)
            blk += nblk
        arr[:, 0:4] = ptrs.view(np.int32)
        dev = ents[0][1][0].device
        self.table = torch.from_numpy(arr).to(dev)
        self.table_n = len(ents)
        self.nblocks = blk

    def get(self, w, K, R, S, C, r0, s0, Ra, Sb, sh, sw):
        if self.pending is not None:   # a prefetched flip writes the cached filters: order after it
            torch.cuda.current_stream(w.device).wait_event(self.pending)
            self.pending = None
        key = (w.data_ptr(), K, R, S, C, r0, s0, Ra, Sb, sh, sw)
        ep = _EPOCH[0]
        ent = self.entries.get(key)
        if ent is not None and ent[0].shape == w.shape:
            if ent[2] != ep:
                if self.table is None or self.table_n != len(self.entries):
                    self._build_table()
                native().flip_weights_batched(self.table, self.table_n, self.nblocks)
                for e in self.entries.values():
                    e[2] = ep
            return ent[1]
        wt = native().flip_weights(w, K, R, S, C, r0, s0, Ra, Sb, sh, sw)
        self.entries[key] = [w, wt, ep]
        self.table = None
        return wt


_PREFETCH = __import__("os").environ.get("ZOO_FLIP_PREFETCH", "1") != "0"


def prefetch_flips(device):
    """Start of a training step: re-flip the cached dgrad filters of every FlatParams on the
    weight-gradient side stream (see _FlipCache.prefetch). No-op under capture."""
    if not (_CACHE_ON and _PREFETCH and _FLATS) or device.type != "cuda" or torch.cuda.is_current_stream_capturing():
        return
    from zoo.ops import wstream
    if not wstream.on():
        return
    side = wstream.side_for(device)
    for ref in list(_FLATS.values()):
        f = ref()
        cache = getattr(f, "_flip_cache", None) if f is not None else None
        if cache is not None and cache.entries and f.bf16.device == device:
            cache.prefetch(side)


_CAPTURE_GEN = [0]


def begin_capture():
    """The training engine is about to capture a step: the first cached filter requested inside
    the capture records ONE batched re-flip of every cached filter into the graph (its replays
    re-flip the weights the replay's own update wrote) instead of one flip launch per conv /
    linear (BERT-base: 0.44 ms of per-layer flips per replay, profiles/r6/bert_b128_graph_critical_r6.md)."""
    _CAPTURE_GEN[0] += 1


def flip_weights(w, K, R, S, C, r0=0, s0=0, Ra=None, Sb=None, sh=1, sw=1):
    Ra, Sb = Ra or R, Sb or S
    cache = _owner_cache(w)
    if cache is not None:
        if not torch.cuda.is_current_stream_capturing():
            return cache.get(w, K, R, S, C, r0, s0, Ra, Sb, sh, sw)
        ent = cache.entries.get((w.data_ptr(), K, R, S, C, r0, s0, Ra, Sb, sh, sw))
        if (ent is not None and ent[0].shape == w.shape and cache.table is not None
                and cache.table_n == len(cache.entries)):
            if cache.cap_gen != _CAPTURE_GEN[0]:
                native().flip_weights_batched(cache.table, cache.table_n, cache.nblocks)
                cache.cap_gen = _CAPTURE_GEN[0]
            return ent[1]
    return native().flip_weights(w, K, R, S, C, r0, s0, Ra, Sb, sh, sw)


# fault injection for the parity tests (tests/test_gpu_native_nets.py): ZOO_FAULT_DGRAD="k:s" scales
# the k-th conv data gradient of the process (0-based, counted from reset_fault_counter) by s --
# proof that a per-layer parity bound catches a 5 % error in ONE layer's backward
_DGRAD_CALLS = [0]


def reset_fault_counter():
    _DGRAD_CALLS[0] = 0


def _fault(dx):
    spec = os.environ.get("ZOO_FAULT_DGRAD")
    if spec:
        k, s = spec.split(":")
        if _DGRAD_CALLS[0] == int(k) and dx is not None:
            dx.mul_(float(s))
        _DGRAD_CALLS[0] += 1
    return dx


def conv_dgrad_s2_compact(dy, wb, K, C):
    """Data gradient of a 1x1 stride-2 unpadded conv in compact form: [N, P, Q, C], the values at
    the even input positions (every other position of the full gradient is zero). Its consumer
    adds it with ``resid_half`` instead of a zero-filled full-size tensor being written."""
    return _fault(conv_fwd(dy, flip_weights(wb, K, 1, 1, C), 1, 1))


def conv_dgrad(dy, wb, K, R, S, C, H, W, stride=(1, 1), pad=(0, 0), dil=(1, 1), resid=None, bstats=None,
               resid_inplace=False, pro=None, resid_half=False):
    """dX [N,H,W,C] of y = conv(x, w) given dY [N,P,Q,K] and the bf16 packed weight.
    ``bstats``: see :func:`conv_fwd` (the result is then the masked dy of the producer).
    ``resid_inplace``: ``resid`` is a temporary the caller gives away; strided dgrads
    with tap-less parity classes accumulate into it instead of a copy of it.
    ``pro``: the BN-backward prologue of :func:`conv_fwd` (stride-1 dgrads; ``dy`` is then the
    masked gradient g of this conv's own BN unit)."""
    return _fault(_conv_dgrad(dy, wb, K, R, S, C, H, W, stride, pad, dil, resid, bstats, resid_inplace, pro,
                              resid_half))


def _conv_dgrad(dy, wb, K, R, S, C, H, W, stride, pad, dil, resid, bstats, resid_inplace, pro=None,
                resid_half=False):
    sh, sw = stride
    if resid_half and not ((sh, sw) == (1, 1) and dil == (1, 1)):
        raise ValueError("conv_dgrad: a half-resolution residual needs a stride-1 dgrad")
    if pro is not None and not ((sh, sw) == (1, 1) or dil != (1, 1)):
        raise ValueError("conv_dgrad: the BN-backward prologue needs a stride-1 dgrad")
    if (sh, sw) == (1, 1) or dil != (1, 1):
        wt = flip_weights(wb, K, R, S, C)
        return conv_fwd(dy, wt, R, S, (1, 1), (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1]), dil, stride,
                        resid=resid, out_hw=(H, W), bstats=bstats, pro=pro, resid_half=resid_half)
    N = dy.shape[0]
    classes = []
    for a in range(sh):
        r0 = (a + pad[0]) % sh
        Ra = (R - r0 + sh - 1) // sh
        Ha = len(range(a, H, sh))
        for b in range(sw):
            s0 = (b + pad[1]) % sw
            Sb = (S - s0 + sw - 1) // sw
            Wb = len(range(b, W, sw))
            if Ha == 0 or Wb == 0:
                continue
            classes.append((a, b, r0, s0, Ra, Sb, Ha, Wb))
    full = all(c[4] > 0 and c[5] > 0 for c in classes) and len(classes) == sh * sw
    if bstats is not None and resid is not None and not full:
        raise NotImplementedError("fused bn-backward with zero parity classes and a residual")
    if resid is not None:
        if full:
            dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dy.device)
        else:
            dx = resid if (resid_inplace and resid.is_contiguous()) else resid.clone()
    else:
        dx = (torch.empty if full else torch.zeros)(N, H, W, C, dtype=torch.bfloat16, device=dy.device)
    for (a, b, r0, s0, Ra, Sb, Ha, Wb) in classes:
        if Ra <= 0 or Sb <= 0:
            continue
        ca = (a + pad[0] - r0) // sh
        cb = (b + pad[1] - s0) // sw
        pa, pb = Ra - 1 - ca, Sb - 1 - cb
        if pa < 0 or pb < 0:  # unusual geometry: fall back to the dilated transposed conv
            wt = flip_weights(wb, K, R, S, C)
            return conv_fwd(dy, wt, R, S, (1, 1), (R - 1 - pad[0], S - 1 - pad[1]), (1, 1), stride, resid=resid,
                            out_hw=(H, W), bstats=bstats)
        wt = flip_weights(wb, K, R, S, C, r0, s0, Ra, Sb, sh, sw)
        # with zero classes dx starts as a copy of resid and is updated in place
        # (the epilogue reads and writes each element from the same lane)
        add = None if resid is None else (resid if full else dx)
        conv_fwd(dy, wt, Ra, Sb, (1, 1), (pa, pb), (1, 1), (1, 1), resid=add, out_hw=(Ha, Wb), out=dx,
                 omap=(H, W, sh, sw, a, b), bstats=bstats)
    # (with bstats, positions no tap reaches stay 0: dy = 0 there and they add nothing to the sums)
    return dx
