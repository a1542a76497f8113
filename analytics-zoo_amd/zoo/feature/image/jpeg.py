"""Batch JPEG decode split CPU / GPU (the serving image path, PreProcessing.scala:24-53):

  * host   csrc/runtime/jpeg.cpp -- marker parsing + Huffman entropy decode of the whole batch
           on C++ threads (GIL released) -> quantised 8x8 DCT blocks + quantisation tables;
  * device csrc/kernels/image.hip -- dequantise + IDCT (one wave per block) -> component
           planes, then chroma upsampling (triangle filter) + YCbCr->RGB fused with the bilinear
           resize / normalise / layout change of the model input.

``decode_resize`` returns None when the batch cannot take this path (progressive / 12-bit /
arithmetic-coded JPEGs, PNGs, mixed geometries); the caller then decodes on the CPU.
``coeffs_to_rgb`` is the numpy twin of the device half (tests)."""
import numpy as np
import torch


def _rt():
    from zoo import _runtime
    return _runtime


def batch_coeffs(payloads, nthreads=8, out=None):
    """Entropy-decode a batch: dict (geometry, coef int16 [N, blocks, 64], qt uint16
    [N, ncomp, 64]) or None. ``out``: a writable int16 numpy buffer (e.g. a pinned host ring
    slot) the coefficients are decoded into when it is large enough."""
    try:
        rt = _rt()
    except ImportError:
        return None
    d = rt.jpeg_batch_coeffs([bytes(p) for p in payloads], int(nthreads), out)
    if d is not None and out is not None:
        n, total = len(payloads), sum(bw * bh for bw, bh in zip(d["bw"], d["bh"]))
        d["coef"] = np.asarray(d["coef"]).reshape(-1)[:n * total * 64].reshape(n, total, 64)
    return d


def geometry(d, n=None):
    nc = d["ncomp"]

    def pad(v, fill):
        v = list(v)
        return v + [fill] * (3 - len(v))
    boff = pad(d["offsets"], d["offsets"][-1] if nc < 3 else 0)
    total = int(d["coef"].shape[1])
    if nc == 1:
        boff = [0, total, total]
    return ([int(n if n is not None else d["coef"].shape[0]), nc, d["w"], d["h"], d["hmax"], d["vmax"]] +
            pad(d["hs"], 1) + pad(d["vs"], 1) + pad(d["bw"], 0) + pad(d["bh"], 0) + boff + [total])


def _to_device(d, device, coef_host=None):
    coef = (coef_host if coef_host is not None else torch.from_numpy(d["coef"])).to(device, non_blocking=True)
    qt = torch.from_numpy(d["qt"].astype(np.int32)).to(device, non_blocking=True)
    return coef, qt


def decode_resize(payloads, out_hw, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0), swap_rb=False, layout=0,
                  device="cuda", nthreads=8):
    """JPEG bytes -> model input on ``device``: layout 0 NCHW fp32, 1 NHWC4 bf16 (the ResNet stem
    input). None if the batch does not qualify for the GPU path."""
    d = batch_coeffs(payloads, nthreads)
    if d is None:
        return None
    return planes_to_input(d, out_hw, mean, std, swap_rb, layout, device)


def planes_to_input(d, out_hw, mean, std, swap_rb, layout, device, coef_host=None):
    """A batch_coeffs() result -> model input on ``device`` (``coef_host``: the pinned tensor
    view of d["coef"], so the upload is one async DMA)."""
    from zoo.ops._native import native
    C = native()
    g = geometry(d)
    coef, qt = _to_device(d, device, coef_host)
    planes = C.jpeg_idct(coef, qt, g)
    return C.jpeg_color_resize(planes, g, int(out_hw[0]), int(out_hw[1]), [float(v) for v in mean],
                               [float(v) for v in std], bool(swap_rb), int(layout))


def decode(payloads, device="cuda", nthreads=8):
    """JPEG bytes -> decoded RGB uint8 [N, H, W, 3] on the device (no resize), or None."""
    d = batch_coeffs(payloads, nthreads)
    if d is None:
        return None
    from zoo.ops._native import native
    C = native()
    g = geometry(d)
    coef, qt = _to_device(d, device)
    planes = C.jpeg_idct(coef, qt, g)
    return C.jpeg_color_resize(planes, g, d["h"], d["w"], [0.0], [1.0], False, 2)


# ---------------------------------------------------------------------------- numpy reference
def _idct_matrix():
    m = np.zeros((8, 8), np.float64)
    for x in range(8):
        for u in range(8):
            m[x, u] = (np.sqrt(0.5) if u == 0 else 1.0) * 0.5 * np.cos((2 * x + 1) * u * np.pi / 16)
    return m


def coeffs_to_rgb(d, i):
    """Image ``i`` of a batch_coeffs() result -> RGB uint8 [H, W, 3] with the device math."""
    M = _idct_matrix()
    w, h, nc = d["w"], d["h"], d["ncomp"]
    planes = []
    for c in range(nc):
        bw, bh, off = d["bw"][c], d["bh"][c], d["offsets"][c]
        blocks = d["coef"][i, off:off + bw * bh].astype(np.float64) * d["qt"][i, c].astype(np.float64)
        blocks = blocks.reshape(bh, bw, 8, 8)
        pix = np.einsum("xu,abvu,yv->abyx", M, blocks, M)
        pix = np.clip(np.rint(pix + 128.0), 0, 255)
        planes.append(pix.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8))
    Y = planes[0][:h, :w]
    if nc == 1:
        return np.repeat(Y[:, :, None], 3, 2).astype(np.uint8)
    hmax, vmax = d["hmax"], d["vmax"]
    chans = []
    for c in (1, 2):
        hs, vs = d["hs"][c], d["vs"][c]
        cw, ch = -(-w * hs // hmax), -(-h * vs // vmax)
        P = planes[c]
        fx = np.clip((np.arange(w) + 0.5) * hs / hmax - 0.5, 0, cw - 1)
        fy = np.clip((np.arange(h) + 0.5) * vs / vmax - 0.5, 0, ch - 1)
        x0, y0 = fx.astype(int), fy.astype(int)
        x1, y1 = np.minimum(x0 + 1, cw - 1), np.minimum(y0 + 1, ch - 1)
        wx, wy = (fx - x0)[None, :], (fy - y0)[:, None]
        top = P[y0][:, x0] + (P[y0][:, x1] - P[y0][:, x0]) * wx
        bot = P[y1][:, x0] + (P[y1][:, x1] - P[y1][:, x0]) * wx
        chans.append(np.rint(top + (bot - top) * wy))
    cb, cr = chans[0] - 128.0, chans[1] - 128.0
    rgb = np.stack([Y + 1.402 * cr, Y - 0.344136286 * cb - 0.714136286 * cr, Y + 1.772 * cb], -1)
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)
