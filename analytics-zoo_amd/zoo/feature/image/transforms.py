"""Image transforms over ImageFeature records (Py/feature/image/imagePreprocessing.py:25-400,
Zs/feature/image/*.scala). A record is a dict: ``uri``, ``bytes`` (encoded),
``mat`` (HWC float32, BGR channel order like the reference's OpenCV Mat),
``originalSize`` (h, w, c), ``label``, ``imageTensor``, ``sample``, ``predict``.

CPU transforms are vectorised numpy; the batch path
(:func:`gpu_resize_normalize`) runs the fused HIP resize + normalize +
layout kernel (csrc/kernels/image.hip) on uint8 batches.
"""
import numpy as np

from zoo.feature.common import Preprocessing

_RNG = np.random.default_rng()


def set_seed(seed):
    global _RNG
    _RNG = np.random.default_rng(seed)


def resize_bilinear(mat, h, w):
    """OpenCV INTER_LINEAR (pixel-centre) resize of an HWC float array."""
    hi, wi = mat.shape[:2]
    if (hi, wi) == (h, w):
        return mat.astype(np.float32, copy=False)
    fy = np.clip((np.arange(h) + 0.5) * (hi / h) - 0.5, 0, hi - 1)
    fx = np.clip((np.arange(w) + 0.5) * (wi / w) - 0.5, 0, wi - 1)
    y0 = fy.astype(np.int64)
    x0 = fx.astype(np.int64)
    y1 = np.minimum(y0 + 1, hi - 1)
    x1 = np.minimum(x0 + 1, wi - 1)
    wy = (fy - y0)[:, None, None].astype(np.float32)
    wx = (fx - x0)[None, :, None].astype(np.float32)
    m = mat.astype(np.float32, copy=False)
    top = m[y0][:, x0] + (m[y0][:, x1] - m[y0][:, x0]) * wx
    bot = m[y1][:, x0] + (m[y1][:, x1] - m[y1][:, x0]) * wx
    return top + (bot - top) * wy


class ImagePreprocessing(Preprocessing):
    def apply(self, feature):
        if isinstance(feature, dict):
            return self.transform(feature)
        return [self.transform(f) for f in feature]

    def transform(self, f):
        raise NotImplementedError


class ImageBytesToMat(ImagePreprocessing):
    def __init__(self, byte_key="bytes", image_codec=-1):
        self.byte_key, self.image_codec = byte_key, image_codec

    def transform(self, f):
        from zoo.pipeline.nnframes.nn_image_reader import decode_image
        arr = decode_image(f[self.byte_key], image_codec=self.image_codec)
        f["mat"] = arr.astype(np.float32)
        f["originalSize"] = arr.shape
        return f


class ImagePixelBytesToMat(ImagePreprocessing):
    def __init__(self, byte_key="bytes"):
        self.byte_key = byte_key

    def transform(self, f):
        h, w, c = f["originalSize"]
        f["mat"] = np.frombuffer(f[self.byte_key], np.uint8).reshape(h, w, c).astype(np.float32)
        return f


class ImageResize(ImagePreprocessing):
    def __init__(self, resize_h, resize_w, resize_mode=1, use_scale_factor=True):
        self.h, self.w = int(resize_h), int(resize_w)

    def transform(self, f):
        f["mat"] = resize_bilinear(f["mat"], self.h, self.w)
        return f


class ImageAspectScale(ImagePreprocessing):
    """Scale the short side to ``min_size`` (capped so the long side <= max_size)."""

    def __init__(self, min_size, scale_multiple_of=1, max_size=1000, resize_mode=1, use_scale_factor=True,
                 min_scale=-1.0):
        self.min_size, self.mult, self.max_size = min_size, scale_multiple_of, max_size

    def _size(self, h, w, target):
        short, long_ = min(h, w), max(h, w)
        scale = target / short
        if round(scale * long_) > self.max_size:
            scale = self.max_size / long_
        nh, nw = int(round(h * scale)), int(round(w * scale))
        if self.mult > 1:
            nh, nw = nh // self.mult * self.mult, nw // self.mult * self.mult
        return max(nh, 1), max(nw, 1)

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        f["mat"] = resize_bilinear(f["mat"], *self._size(h, w, self.min_size))
        return f


class ImageRandomAspectScale(ImageAspectScale):
    def __init__(self, scales, scale_multiple_of=1, max_size=1000):
        super().__init__(scales[0], scale_multiple_of, max_size)
        self.scales = list(scales)

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        f["mat"] = resize_bilinear(f["mat"], *self._size(h, w, self.scales[_RNG.integers(len(self.scales))]))
        return f


class ImageBrightness(ImagePreprocessing):
    def __init__(self, delta_low, delta_high):
        self.lo, self.hi = delta_low, delta_high

    def transform(self, f):
        f["mat"] = f["mat"] + _RNG.uniform(self.lo, self.hi)
        return f


class ImageContrast(ImagePreprocessing):
    def __init__(self, delta_low, delta_high):
        self.lo, self.hi = delta_low, delta_high

    def transform(self, f):
        f["mat"] = f["mat"] * _RNG.uniform(self.lo, self.hi)
        return f


def _bgr_to_hsv(m):
    b, g, r = m[..., 0] / 255.0, m[..., 1] / 255.0, m[..., 2] / 255.0
    mx, mn = np.maximum(np.maximum(r, g), b), np.minimum(np.minimum(r, g), b)
    d = mx - mn
    h = np.zeros_like(mx)
    nz = d > 1e-12
    rm = nz & (mx == r)
    gm = nz & (mx == g) & ~rm
    bm = nz & ~rm & ~gm
    h[rm] = (60 * ((g - b)[rm] / d[rm])) % 360
    h[gm] = 60 * ((b - r)[gm] / d[gm]) + 120
    h[bm] = 60 * ((r - g)[bm] / d[bm]) + 240
    s = np.where(mx > 1e-12, d / np.maximum(mx, 1e-12), 0)
    return h, s, mx


def _hsv_to_bgr(h, s, v):
    c = v * s
    hp = (h % 360) / 60.0
    x = c * (1 - np.abs(hp % 2 - 1))
    z = np.zeros_like(h)
    conds = [(hp < 1), (hp < 2), (hp < 3), (hp < 4), (hp < 5), (hp >= 5)]
    rgb = [(c, x, z), (x, c, z), (z, c, x), (z, x, c), (x, z, c), (c, z, x)]
    r = np.select(conds, [t[0] for t in rgb])
    g = np.select(conds, [t[1] for t in rgb])
    b = np.select(conds, [t[2] for t in rgb])
    m = v - c
    return np.stack([(b + m), (g + m), (r + m)], -1) * 255.0


class ImageHue(ImagePreprocessing):
    def __init__(self, delta_low, delta_high):
        self.lo, self.hi = delta_low, delta_high

    def transform(self, f):
        h, s, v = _bgr_to_hsv(f["mat"])
        f["mat"] = _hsv_to_bgr(h + _RNG.uniform(self.lo, self.hi), s, v).astype(np.float32)
        return f


class ImageSaturation(ImagePreprocessing):
    def __init__(self, delta_low, delta_high):
        self.lo, self.hi = delta_low, delta_high

    def transform(self, f):
        h, s, v = _bgr_to_hsv(f["mat"])
        f["mat"] = _hsv_to_bgr(h, np.clip(s * _RNG.uniform(self.lo, self.hi), 0, 1), v).astype(np.float32)
        return f


class ImageColorJitter(ImagePreprocessing):
    def __init__(self, brightness_prob=0.5, brightness_delta=32.0, contrast_prob=0.5, contrast_lower=0.5,
                 contrast_upper=1.5, hue_prob=0.5, hue_delta=18.0, saturation_prob=0.5, saturation_lower=0.5,
                 saturation_upper=1.5, random_order_prob=0.0, shuffle=False):
        self.ops = [(brightness_prob, ImageBrightness(-brightness_delta, brightness_delta)),
                    (contrast_prob, ImageContrast(contrast_lower, contrast_upper)),
                    (saturation_prob, ImageSaturation(saturation_lower, saturation_upper)),
                    (hue_prob, ImageHue(-hue_delta, hue_delta))]
        self.random_order_prob = random_order_prob

    def transform(self, f):
        ops = list(self.ops)
        if _RNG.random() < self.random_order_prob:
            _RNG.shuffle(ops)
        for p, op in ops:
            if _RNG.random() < p:
                f = op.transform(f)
        return f


class ImageChannelNormalize(ImagePreprocessing):
    """(x - mean) / std per channel; arguments in R, G, B order, the Mat is BGR."""

    def __init__(self, mean_r, mean_g, mean_b, std_r=1.0, std_g=1.0, std_b=1.0):
        self.mean = np.array([mean_b, mean_g, mean_r], np.float32)
        self.std = np.array([std_b, std_g, std_r], np.float32)

    def transform(self, f):
        f["mat"] = (f["mat"] - self.mean) / self.std
        return f


class ImageChannelScaledNormalizer(ImagePreprocessing):
    def __init__(self, mean_r, mean_g, mean_b, scale):
        self.mean = np.array([mean_b, mean_g, mean_r], np.float32)
        self.scale = scale

    def transform(self, f):
        f["mat"] = (f["mat"] - self.mean) * self.scale
        return f


class PerImageNormalize(ImagePreprocessing):
    def __init__(self, min=0.0, max=1.0, norm_type=32):  # noqa: A002
        self.lo, self.hi = min, max

    def transform(self, f):
        m = f["mat"]
        mn, mx = m.min(), m.max()
        f["mat"] = (m - mn) / max(mx - mn, 1e-12) * (self.hi - self.lo) + self.lo
        return f


class ImagePixelNormalize(ImagePreprocessing):
    def __init__(self, means):
        self.means = np.asarray(means, np.float32)

    def transform(self, f):
        f["mat"] = f["mat"] - self.means.reshape(f["mat"].shape)
        return f


class _Crop(ImagePreprocessing):
    def _crop(self, f, x1, y1, x2, y2):
        h, w = f["mat"].shape[:2]
        x1, y1 = max(0, int(x1)), max(0, int(y1))
        x2, y2 = min(w, int(x2)), min(h, int(y2))
        f["mat"] = f["mat"][y1:y2, x1:x2]
        # the crop window in normalised coordinates of the pre-crop image (ImageRoiProject)
        f["cropBbox"] = np.array([x1 / w, y1 / h, x2 / w, y2 / h], np.float32)
        return f


class ImageCenterCrop(_Crop):
    def __init__(self, crop_width, crop_height, is_clip=True):
        self.cw, self.ch = crop_width, crop_height

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        x1, y1 = (w - self.cw) // 2, (h - self.ch) // 2
        return self._crop(f, x1, y1, x1 + self.cw, y1 + self.ch)


class ImageRandomCrop(_Crop):
    def __init__(self, crop_width, crop_height, is_clip=True):
        self.cw, self.ch = crop_width, crop_height

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        x1 = _RNG.integers(0, max(w - self.cw, 0) + 1)
        y1 = _RNG.integers(0, max(h - self.ch, 0) + 1)
        return self._crop(f, x1, y1, x1 + self.cw, y1 + self.ch)


class ImageFixedCrop(_Crop):
    def __init__(self, x1, y1, x2, y2, normalized=True, is_clip=True):
        self.box, self.normalized = (x1, y1, x2, y2), normalized

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        x1, y1, x2, y2 = self.box
        if self.normalized:
            x1, x2, y1, y2 = x1 * w, x2 * w, y1 * h, y2 * h
        return self._crop(f, x1, y1, x2, y2)


class ImageExpand(ImagePreprocessing):
    """Place the image on a larger mean-filled canvas (SSD zoom-out)."""

    def __init__(self, means_r=123, means_g=117, means_b=104, min_expand_ratio=1.0, max_expand_ratio=4.0):
        self.means = np.array([means_b, means_g, means_r], np.float32)
        self.lo, self.hi = min_expand_ratio, max_expand_ratio

    def transform(self, f):
        m = f["mat"]
        h, w, c = m.shape
        r = _RNG.uniform(self.lo, self.hi)
        nh, nw = int(h * r), int(w * r)
        top, left = _RNG.integers(0, nh - h + 1), _RNG.integers(0, nw - w + 1)
        out = np.empty((nh, nw, c), np.float32)
        out[...] = self.means[:c]
        out[top:top + h, left:left + w] = m
        f["mat"] = out
        f["expand"] = (top, left, r)
        return f


class ImageFiller(ImagePreprocessing):
    def __init__(self, start_x, start_y, end_x, end_y, value=255):
        self.box, self.value = (start_x, start_y, end_x, end_y), value

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        x1, y1, x2, y2 = self.box
        f["mat"][int(y1 * h):int(y2 * h), int(x1 * w):int(x2 * w)] = self.value
        return f


class ImageHFlip(ImagePreprocessing):
    def transform(self, f):
        f["mat"] = f["mat"][:, ::-1].copy()
        return f


ImageMirror = ImageHFlip


class ImageChannelOrder(ImagePreprocessing):
    """Random permutation of the channels (data augmentation)."""

    def transform(self, f):
        f["mat"] = f["mat"][..., _RNG.permutation(f["mat"].shape[2])]
        return f


class ImageMatToTensor(ImagePreprocessing):
    def __init__(self, to_RGB=False, tensor_key="imageTensor", share_buffer=True, format="NCHW"):  # noqa: A002,N803
        self.to_rgb, self.key, self.format = to_RGB, tensor_key, format

    def transform(self, f):
        m = f["mat"]
        if self.to_rgb and m.shape[2] >= 3:
            m = m[..., [2, 1, 0] + list(range(3, m.shape[2]))]
        f[self.key] = np.ascontiguousarray(m.transpose(2, 0, 1) if self.format == "NCHW" else m, np.float32)
        return f


class ImageMatToFloats(ImageMatToTensor):
    def __init__(self, valid_height=300, valid_width=300, valid_channel=3, out_key="floats", share_buffer=True):
        super().__init__(False, out_key, share_buffer, "NHWC")


class ImageSetToSample(ImagePreprocessing):
    def __init__(self, input_keys=("imageTensor",), target_keys=("label",), sample_key="sample"):
        self.inputs, self.targets, self.key = list(input_keys), list(target_keys or []), sample_key

    def transform(self, f):
        feats = [f[k] for k in self.inputs]
        labels = [np.asarray(f[k], np.float32) for k in self.targets if k in f]
        f[self.key] = (feats[0] if len(feats) == 1 else feats, labels[0] if len(labels) == 1 else
                       (labels or None))
        return f


class ImageFeatureToTensor(Preprocessing):
    def apply(self, f):
        return f["imageTensor"]


class ImageFeatureToSample(Preprocessing):
    def apply(self, f):
        return (f["imageTensor"], f.get("label"))


class RowToImageFeature(Preprocessing):
    """NNImageReader row (Spark-image struct dict) -> ImageFeature."""

    def apply(self, row):
        from zoo.pipeline.nnframes.nn_image_reader import row_to_array
        arr = row_to_array(row)
        return {"uri": row.get("origin"), "mat": arr.astype(np.float32), "originalSize": arr.shape}


class ImageRandomPreprocessing(ImagePreprocessing):
    def __init__(self, preprocessing, prob):
        self.p, self.prob = preprocessing, prob

    def transform(self, f):
        return self.p.transform(f) if _RNG.random() < self.prob else f


def gpu_resize_normalize(batch_u8, out_h, out_w, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0), swap_rb=False,
                         layout="NCHW", device="cuda"):
    """uint8 [N, H, W, C] -> fused HIP resize + normalize (+ BGR<->RGB) on the GPU.
    ``layout``: "NCHW" (fp32) or "NHWC4" (bf16, channels zero-padded to 4 — the
    ResNet stem's input format)."""
    import torch
    from zoo.ops._native import native
    t = torch.as_tensor(np.ascontiguousarray(batch_u8, dtype=np.uint8)).to(device, non_blocking=True)
    return native().resize_normalize(t, int(out_h), int(out_w), [float(m) for m in mean], [float(s) for s in std],
                                     bool(swap_rb), 0 if layout == "NCHW" else 1)


# ---------------------------------------------------------------------------
# Random cropper and region-of-interest transformers
# (Zs/feature/image/ImageRandomCropper.scala, RoiTransformer.scala, RandomSampler.scala)
#
# A feature's ground-truth boxes live in ``f["roi"]`` = {"classes": [n] (or [2, n] with the
# difficult flags as row 1), "bboxes": [n, 4] float (x1, y1, x2, y2)} -- BigDL's RoiLabel.
# ---------------------------------------------------------------------------
def _roi(f):
    r = f.get("roi")
    if r is None and isinstance(f.get("label"), dict):
        r = f["roi"] = f["label"]
    return r


class ImageRandomCropper(_Crop):
    """Crop ``crop_width`` x ``crop_height`` at a random (``cropper_method="random"``) or
    centred position, then mirror horizontally with probability 1/2 when ``mirror``."""

    def __init__(self, crop_width, crop_height, mirror=False, cropper_method="random", channels=3):
        self.cw, self.ch = int(crop_width), int(crop_height)
        self.mirror, self.method, self.channels = bool(mirror), str(cropper_method).lower(), int(channels)

    def transform(self, f):
        h, w = f["mat"].shape[:2]
        if self.method in ("random", "croprandom"):
            x1 = int(_RNG.integers(0, max(w - self.cw, 0) + 1))
            y1 = int(_RNG.integers(0, max(h - self.ch, 0) + 1))
        else:
            x1, y1 = max(w - self.cw, 0) // 2, max(h - self.ch, 0) // 2
        f = self._crop(f, x1, y1, x1 + self.cw, y1 + self.ch)
        if self.mirror and _RNG.random() < 0.5:
            f["mat"] = f["mat"][:, ::-1].copy()
        return f


class ImageRoiNormalize(ImagePreprocessing):
    """Boxes from pixels to [0, 1] of the current image size."""

    def transform(self, f):
        r = _roi(f)
        if r is not None and len(r["bboxes"]):
            h, w = f["mat"].shape[:2]
            r["bboxes"] = np.asarray(r["bboxes"], np.float32) / np.array([w, h, w, h], np.float32)
        return f


class ImageRoiHFlip(ImagePreprocessing):
    """Mirror the boxes horizontally (pair with ImageHFlip)."""

    def __init__(self, normalized=True):
        self.normalized = normalized

    def transform(self, f):
        r = _roi(f)
        if r is not None and len(r["bboxes"]):
            b = np.asarray(r["bboxes"], np.float32).copy()
            width = 1.0 if self.normalized else float(f["mat"].shape[1])
            x1 = width - b[:, 2]
            b[:, 2] = width - b[:, 0]
            b[:, 0] = x1
            r["bboxes"] = b
        return f


class ImageRoiResize(ImagePreprocessing):
    """Scale pixel boxes by the resize from ``originalSize`` to the current size (a no-op
    for normalised boxes)."""

    def __init__(self, normalized=False):
        self.normalized = normalized

    def transform(self, f):
        r = _roi(f)
        if r is not None and len(r["bboxes"]) and not self.normalized:
            oh, ow = f["originalSize"][:2]
            h, w = f["mat"].shape[:2]
            r["bboxes"] = np.asarray(r["bboxes"], np.float32) * np.array([w / ow, h / oh, w / ow, h / oh],
                                                                          np.float32)
        return f


class ImageRoiProject(ImagePreprocessing):
    """Project normalised boxes onto the last crop window (``f["cropBbox"]``): boxes whose
    centre falls outside the window are dropped when ``need_meet_center_constraint``, the
    rest are clipped to the window and re-normalised to it; empty boxes are dropped."""

    def __init__(self, need_meet_center_constraint=True):
        self.center = need_meet_center_constraint

    def transform(self, f):
        r = _roi(f)
        crop = f.get("cropBbox")
        if r is None or crop is None or not len(r["bboxes"]):
            return f
        b = np.asarray(r["bboxes"], np.float32)
        cx1, cy1, cx2, cy2 = [float(v) for v in crop]
        keep = np.ones(len(b), bool)
        if self.center:
            mx, my = (b[:, 0] + b[:, 2]) / 2, (b[:, 1] + b[:, 3]) / 2
            keep &= (mx >= cx1) & (mx <= cx2) & (my >= cy1) & (my <= cy2)
        cw, ch = max(cx2 - cx1, 1e-12), max(cy2 - cy1, 1e-12)
        nb = np.stack([(np.clip(b[:, 0], cx1, cx2) - cx1) / cw, (np.clip(b[:, 1], cy1, cy2) - cy1) / ch,
                       (np.clip(b[:, 2], cx1, cx2) - cx1) / cw, (np.clip(b[:, 3], cy1, cy2) - cy1) / ch], 1)
        keep &= (nb[:, 2] > nb[:, 0]) & (nb[:, 3] > nb[:, 1])
        r["bboxes"] = nb[keep]
        cls = np.asarray(r["classes"])
        r["classes"] = cls[..., keep] if cls.ndim == 2 else cls[keep]
        return f


def _iou(box, boxes):
    ix1 = np.maximum(box[0], boxes[:, 0])
    iy1 = np.maximum(box[1], boxes[:, 1])
    ix2 = np.minimum(box[2], boxes[:, 2])
    iy2 = np.minimum(box[3], boxes[:, 3])
    inter = np.clip(ix2 - ix1, 0, None) * np.clip(iy2 - iy1, 0, None)
    area = (box[2] - box[0]) * (box[3] - box[1]) + (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    return inter / np.maximum(area - inter, 1e-12)


class ImageRandomSampler(_Crop):
    """SSD batch sampler (RandomSampler.scala): among the whole image and crops drawn by
    samplers (scale in [0.3, 1], aspect ratio in [0.5, 2], up to 50 trials each) that reach
    a minimum Jaccard overlap of {0.1, 0.3, 0.5, 0.7, 0.9} or any with a ground-truth box,
    one is picked at random and cropped; follow with ImageRoiProject for the boxes."""

    MIN_IOU = (None, 0.1, 0.3, 0.5, 0.7, 0.9, "max")

    def __init__(self, max_trials=50, min_scale=0.3, max_scale=1.0, min_ar=0.5, max_ar=2.0):
        self.max_trials, self.min_scale, self.max_scale = max_trials, min_scale, max_scale
        self.min_ar, self.max_ar = min_ar, max_ar

    def _sample_box(self):
        scale = _RNG.uniform(self.min_scale, self.max_scale)
        ar = _RNG.uniform(max(self.min_ar, scale ** 2), min(self.max_ar, 1.0 / scale ** 2))
        bw, bh = scale * np.sqrt(ar), scale / np.sqrt(ar)
        x1, y1 = _RNG.uniform(0, 1 - bw), _RNG.uniform(0, 1 - bh)
        return np.array([x1, y1, x1 + bw, y1 + bh], np.float32)

    def transform(self, f):
        r = _roi(f)
        gt = np.asarray(r["bboxes"], np.float32) if r is not None and len(r["bboxes"]) else None
        cands = [np.array([0, 0, 1, 1], np.float32)]
        for thr in self.MIN_IOU[1:]:
            for _ in range(self.max_trials):
                box = self._sample_box()
                if gt is None:
                    cands.append(box)
                    break
                ious = _iou(box, gt)
                if (thr == "max" and ious.max() >= 1.0) or (thr != "max" and ious.max() >= thr):
                    cands.append(box)
                    break
        box = cands[int(_RNG.integers(0, len(cands)))]
        h, w = f["mat"].shape[:2]
        return self._crop(f, box[0] * w, box[1] * h, box[2] * w, box[3] * h)
