"""3D image (volume) transforms (Zs/feature/image3d/*.scala: Crop3D, Rotate3D,
AffineTransform3D, Warp; Py/feature/image3d/transformation.py).

Volumes are [D, H, W] or [D, H, W, C] float arrays in an ImageFeature3D
dict (key ``image``). Affine resampling uses trilinear interpolation through
``torch.nn.functional.grid_sample`` (runs on the GPU when the volume is on one).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from zoo.feature.common import Preprocessing


def ImageFeature3D(image, label=None, uri=None):  # noqa: N802 - reference name
    f = {"image": np.asarray(image, np.float32), "uri": uri}
    if label is not None:
        f["label"] = label
    return f


class _T3(Preprocessing):
    def apply(self, f):
        if isinstance(f, dict):
            return self.transform(f)
        return [self.transform(x) for x in f]


class Crop3D(_T3):
    def __init__(self, start, patch_size):
        self.start, self.size = list(start), list(patch_size)

    def transform(self, f):
        (z, y, x), (d, h, w) = self.start, self.size
        f["image"] = f["image"][z:z + d, y:y + h, x:x + w]
        return f


class RandomCrop3D(Crop3D):
    def __init__(self, crop_depth, crop_height, crop_width, seed=None):
        super().__init__([0, 0, 0], [crop_depth, crop_height, crop_width])
        self.rng = np.random.default_rng(seed)

    def transform(self, f):
        D, H, W = f["image"].shape[:3]
        self.start = [self.rng.integers(0, max(D - self.size[0], 0) + 1),
                      self.rng.integers(0, max(H - self.size[1], 0) + 1),
                      self.rng.integers(0, max(W - self.size[2], 0) + 1)]
        return super().transform(f)


class CenterCrop3D(Crop3D):
    def __init__(self, crop_depth, crop_height, crop_width):
        super().__init__([0, 0, 0], [crop_depth, crop_height, crop_width])

    def transform(self, f):
        D, H, W = f["image"].shape[:3]
        self.start = [(D - self.size[0]) // 2, (H - self.size[1]) // 2, (W - self.size[2]) // 2]
        return super().transform(f)


def _resample(vol, mat, translation=(0.0, 0.0, 0.0), clamp_mode="clamp", pad_val=0.0):
    """out[p] = vol[mat @ (p - c) + c + t] with voxel coordinates (z, y, x), trilinear."""
    v = torch.as_tensor(vol, dtype=torch.float32)
    chan_last = v.dim() == 4
    if not chan_last:
        v = v[..., None]
    D, H, W, C = v.shape
    dev = v.device
    zz, yy, xx = torch.meshgrid(torch.arange(D, device=dev, dtype=torch.float32),
                                torch.arange(H, device=dev, dtype=torch.float32),
                                torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    c = torch.tensor([(D - 1) / 2, (H - 1) / 2, (W - 1) / 2], device=dev)
    p = torch.stack([zz, yy, xx], -1) - c
    m = torch.as_tensor(np.asarray(mat, np.float32), device=dev)
    src = p @ m.t() + c + torch.as_tensor(translation, dtype=torch.float32, device=dev)
    # grid_sample wants (x, y, z) normalised to [-1, 1]
    norm = torch.stack([src[..., 2] / max(W - 1, 1), src[..., 1] / max(H - 1, 1), src[..., 0] / max(D - 1, 1)],
                       -1) * 2 - 1
    inp = v.permute(3, 0, 1, 2)[None]
    mode = "border" if clamp_mode == "clamp" else "zeros"
    out = F.grid_sample(inp - pad_val if mode == "zeros" else inp, norm[None], mode="bilinear",
                        padding_mode=mode, align_corners=True)
    if mode == "zeros":
        out = out + pad_val
    out = out[0].permute(1, 2, 3, 0)
    out = out if chan_last else out[..., 0]
    return out.cpu().numpy() if not torch.is_tensor(vol) else out


class AffineTransform3D(_T3):
    def __init__(self, mat, translation=(0.0, 0.0, 0.0), clamp_mode="clamp", pad_val=0.0):
        self.mat, self.t, self.mode, self.pad = np.asarray(mat, np.float32), translation, clamp_mode, pad_val

    def transform(self, f):
        f["image"] = _resample(f["image"], self.mat, self.t, self.mode, self.pad)
        return f


class Rotate3D(AffineTransform3D):
    """Rotation by (yaw, pitch, roll) radians about the volume centre."""

    def __init__(self, rotation_angles):
        a, b, g = rotation_angles
        rz = np.array([[1, 0, 0], [0, math.cos(a), -math.sin(a)], [0, math.sin(a), math.cos(a)]])
        ry = np.array([[math.cos(b), 0, math.sin(b)], [0, 1, 0], [-math.sin(b), 0, math.cos(b)]])
        rx = np.array([[math.cos(g), -math.sin(g), 0], [math.sin(g), math.cos(g), 0], [0, 0, 1]])
        super().__init__(rz @ ry @ rx)


class Warp(_T3):
    """Displace every voxel by a flow field [D, H, W, 3] (dz, dy, dx)."""

    def __init__(self, flow, offset=True, clamp_mode="clamp", pad_val=0.0):
        self.flow, self.mode, self.pad = np.asarray(flow, np.float32), clamp_mode, pad_val

    def transform(self, f):
        vol = torch.as_tensor(f["image"], dtype=torch.float32)
        D, H, W = vol.shape[:3]
        zz, yy, xx = torch.meshgrid(torch.arange(D, dtype=torch.float32), torch.arange(H, dtype=torch.float32),
                                    torch.arange(W, dtype=torch.float32), indexing="ij")
        fl = torch.as_tensor(self.flow)
        src = torch.stack([zz, yy, xx], -1) + fl
        norm = torch.stack([src[..., 2] / max(W - 1, 1), src[..., 1] / max(H - 1, 1), src[..., 0] / max(D - 1, 1)],
                           -1) * 2 - 1
        v = vol if vol.dim() == 4 else vol[..., None]
        out = F.grid_sample(v.permute(3, 0, 1, 2)[None], norm[None], mode="bilinear",
                            padding_mode="border" if self.mode == "clamp" else "zeros", align_corners=True)
        out = out[0].permute(1, 2, 3, 0)
        f["image"] = (out if vol.dim() == 4 else out[..., 0]).numpy()
        return f
