"""Split JPEG decoder: the C++ baseline entropy decoder (csrc/runtime/jpeg.cpp) feeding the
HIP IDCT / upsample / colour / resize kernels (image.hip). CPU: entropy decode + the numpy twin
of the device math reproduce PIL's libjpeg decode within JPEG rounding (+-3, mean < 0.25) for
4:2:0 / 4:2:2 / 4:4:4 / grayscale, restart intervals, odd sizes; unsupported streams
(progressive, PNG) return None. GPU: the kernels equal the numpy twin and the fused resize
equals resize_normalize of the decoded image."""
import io

import numpy as np
import pytest
from PIL import Image

jpeg = pytest.importorskip("zoo.feature.image.jpeg")


def _img(h, w, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    a = np.stack([xx * 255 // max(1, w - 1), yy * 255 // max(1, h - 1), (xx + yy) * 3 % 256], -1).astype(float)
    return np.clip(a + rng.normal(0, 20, a.shape), 0, 255).astype(np.uint8)


def _enc(a, gray=False, **kw):
    b = io.BytesIO()
    Image.fromarray(a[:, :, 0] if gray else a, "L" if gray else "RGB").save(b, "JPEG", quality=90, **kw)
    return b.getvalue()


CASES = [((64, 80), dict(subsampling=2)), ((61, 77), dict(subsampling=0)), ((48, 50), dict(subsampling=1)),
         ((37, 29), dict(gray=True)), ((256, 256), dict(subsampling=2, restart_marker_blocks=3)),
         ((96, 128), dict(subsampling=2, restart_marker_rows=1))]


@pytest.mark.parametrize("hw,kw", CASES)
def test_entropy_decode_matches_pil(hw, kw):
    p = _enc(_img(*hw), **kw)
    d = jpeg.batch_coeffs([p, p], nthreads=2)
    assert d is not None and d["w"] == hw[1] and d["h"] == hw[0]
    ref = np.asarray(Image.open(io.BytesIO(p)).convert("RGB")).astype(int)
    for i in range(2):
        diff = np.abs(jpeg.coeffs_to_rgb(d, i).astype(int) - ref)
        assert diff.max() <= 3 and diff.mean() < 0.25, (diff.max(), diff.mean())


def test_unsupported_streams_fall_back():
    a = _img(32, 32)
    b = io.BytesIO()
    Image.fromarray(a).save(b, "JPEG", progressive=True)
    assert jpeg.batch_coeffs([b.getvalue()]) is None
    b = io.BytesIO()
    Image.fromarray(a).save(b, "PNG")
    assert jpeg.batch_coeffs([b.getvalue()]) is None
    # mixed geometries in one batch -> None (the caller decodes on the CPU)
    assert jpeg.batch_coeffs([_enc(_img(32, 32)), _enc(_img(40, 32))]) is None
    # truncated stream
    assert jpeg.batch_coeffs([_enc(_img(32, 32))[:200]]) is None


def test_malformed_huffman_table_is_rejected():
    """an over-subscribed DHT (255 codes of length 1) must be rejected before the
    10-bit lookup table is filled (it used to write ~256 KB past it)."""
    good = _enc(_img(32, 32))
    counts = bytes([255] + [0] * 15)
    vals = bytes(range(255))
    seg = b"\xff\xc4" + (2 + 17 + len(vals)).to_bytes(2, "big") + b"\x00" + counts + vals
    bad = good[:2] + seg + good[2:]
    for _ in range(3):
        assert jpeg.batch_coeffs([bad]) is None
    # a code space over-subscribed only at a later length (2 codes of len 1 + 1 of len 2)
    counts = bytes([2, 1] + [0] * 14)
    seg = b"\xff\xc4" + (2 + 17 + 3).to_bytes(2, "big") + b"\x10" + counts + b"\x00\x01\x02"
    assert jpeg.batch_coeffs([good[:2] + seg + good[2:]]) is None
    assert jpeg.batch_coeffs([good]) is not None


def test_second_frame_header_after_a_scan_is_rejected():
    """a second SOF after the first scan (larger geometry) must not re-size the block
    grid of a caller-provided destination: the decode fails before any scan writes."""
    good = _enc(_img(16, 16))
    big = _enc(_img(512, 512))
    i_sof = big.index(b"\xff\xc0")
    sof_len = int.from_bytes(big[i_sof + 2:i_sof + 4], "big")
    sof = big[i_sof:i_sof + 2 + sof_len]
    i_sos = big.index(b"\xff\xda")
    tail = big[i_sos:]                               # the big image's scan + EOI
    evil = good[:-2] + sof + tail
    d = jpeg.batch_coeffs([good], nthreads=1)
    out = np.zeros((1,) + d["coef"].shape[1:], np.int16)
    assert jpeg.batch_coeffs([evil], nthreads=1, out=out) is None


@pytest.mark.gpu
@pytest.mark.parametrize("hw,kw", CASES)
def test_gpu_decode_matches_reference(gpu, hw, kw):
    import torch
    p = _enc(_img(*hw, seed=1), **kw)
    out = jpeg.decode([p, p], device=gpu)
    d = jpeg.batch_coeffs([p, p])
    ref = jpeg.coeffs_to_rgb(d, 0).astype(int)
    got = out.cpu().numpy().astype(int)
    assert got.shape == (2, hw[0], hw[1], 3)
    # fp32 device math vs the fp64 twin: a chroma sample on a rounding boundary moves by 1 and
    # the 1.772 / 1.402 YCbCr coefficients carry that to a 2 in R or B
    assert np.abs(got[0] - ref).max() <= 2 and (got[0] != ref).mean() < 0.01
    assert torch.equal(out[0], out[1])


@pytest.mark.gpu
def test_gpu_decode_resize_matches_resize_normalize(gpu):
    import torch
    from zoo.ops._native import native
    p = _enc(_img(200, 240, seed=2), subsampling=2)
    mean, std = [123.7, 116.3, 103.5], [58.4, 57.1, 57.4]
    rgb = jpeg.decode([p] * 3, device=gpu)
    for layout in (0, 1):
        fused = jpeg.decode_resize([p] * 3, (224, 224), mean, std, swap_rb=False, layout=layout, device=gpu)
        ref = native().resize_normalize(rgb.contiguous(), 224, 224, mean, std, False, layout)
        assert fused.shape == ref.shape
        torch.testing.assert_close(fused.float(), ref.float(), atol=2e-2, rtol=1e-2)
