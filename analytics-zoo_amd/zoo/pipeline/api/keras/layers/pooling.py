"""Pooling layers (Py/pipeline/api/keras/layers/pooling.py; Zs MaxPooling1D/2D/3D,
AveragePooling1D/2D/3D, GlobalMax/AveragePooling1D/2D/3D).

2-D max pooling and global average pooling on channels-last inputs with
8-aligned channels run on the native NHWC kernels (byte-argmax max pooling);
everything else uses PyTorch-ROCm pooling.
"""
import math

import torch
import torch.nn.functional as F

from zoo import ops
from zoo.pipeline.api.keras.base import Layer


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)


def _pool_out(size, k, s, mode):
    if size is None:
        return None
    if mode == "same":
        return int(math.ceil(size / s))
    return (size - k) // s + 1


def _same_pad(size, k, s):
    out = int(math.ceil(size / s))
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


class _Pool2D(Layer):
    kind = "max"

    def __init__(self, pool_size=(2, 2), strides=None, border_mode="valid", dim_ordering="th", input_shape=None,
                 pads=None, count_include_pad=True, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.border_mode, self.dim_ordering = border_mode, dim_ordering
        self.count_include_pad = count_include_pad

    def compute_output_shape(self, s):
        hw = (s[2], s[3]) if self.dim_ordering == "th" else (s[1], s[2])
        o = [_pool_out(hw[i], self.pool_size[i], self.strides[i], self.border_mode) for i in range(2)]
        return (None, s[1], o[0], o[1]) if self.dim_ordering == "th" else (None, o[0], o[1], s[3])

    def _pad_nchw(self, x):
        if self.border_mode != "same":
            return x, (0, 0)
        ph = _same_pad(x.shape[2], self.pool_size[0], self.strides[0])
        pw = _same_pad(x.shape[3], self.pool_size[1], self.strides[1])
        if ph[0] == ph[1] and pw[0] == pw[1]:
            return x, (ph[0], pw[0])
        fill = float("-inf") if self.kind == "max" else 0.0
        return F.pad(x, (pw[0], pw[1], ph[0], ph[1]), value=fill), (0, 0)

    def _native(self, xn):
        """NHWC x -> NHWC pooled on the native kernels; None if the geometry is unsupported."""
        pad = (0, 0)
        if self.border_mode == "same":
            ph = _same_pad(xn.shape[1], self.pool_size[0], self.strides[0])
            pw = _same_pad(xn.shape[2], self.pool_size[1], self.strides[1])
            if ph[0] != ph[1] or pw[0] != pw[1]:
                return None
            pad = (ph[0], pw[0])
        if self.kind == "max":
            return ops.max_pool2d_nhwc(xn, self.pool_size, self.strides, pad)
        from zoo.ops.pool import avg_pool2d_nhwc
        if 2 * pad[0] > self.pool_size[0] or 2 * pad[1] > self.pool_size[1]:
            return None
        return avg_pool2d_nhwc(xn, self.pool_size, self.strides, pad, count_include_pad=self.count_include_pad)

    def call(self, x):
        if x.is_cuda and x.dim() == 4:
            th = self.dim_ordering == "th"
            xn = x.permute(0, 2, 3, 1) if th else x
            c = xn.shape[-1]
            xp = xn if c % 8 == 0 else F.pad(xn, (0, (-c) % 8))  # the kernels move 8 channels per lane
            y = self._native(xp.contiguous())
            if y is not None:
                y = y.to(x.dtype)[..., :c]
                return y.permute(0, 3, 1, 2) if th else y
        xc = x if self.dim_ordering == "th" else x.permute(0, 3, 1, 2)
        xc, pad = self._pad_nchw(xc)
        if self.kind == "max":
            y = F.max_pool2d(xc, self.pool_size, self.strides, pad)
        else:
            y = F.avg_pool2d(xc, self.pool_size, self.strides, pad, count_include_pad=self.count_include_pad)
        return y if self.dim_ordering == "th" else y.permute(0, 2, 3, 1).contiguous()


class MaxPooling2D(_Pool2D):
    kind = "max"


class AveragePooling2D(_Pool2D):
    kind = "avg"


class _Pool1D(Layer):
    kind = "max"

    def __init__(self, pool_length=2, stride=None, border_mode="valid", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.pool_length = int(pool_length)
        self.stride = int(stride) if stride is not None else self.pool_length
        self.border_mode = border_mode

    def compute_output_shape(self, s):
        return (None, _pool_out(s[1], self.pool_length, self.stride, self.border_mode), s[2])

    def call(self, x):
        from zoo.ops.layers import pool1d_nwc
        pad = (0, 0)
        if self.border_mode == "same":
            pad = tuple(_same_pad(x.shape[1], self.pool_length, self.stride))
        if x.is_cuda and pad != (0, 0) and x.shape[-1] % 8 == 0:
            # explicit edge padding (-inf for max, 0 for average as the reference does), then
            # the native pool with no implicit padding
            x = F.pad(x, (0, 0, pad[0], pad[1]), value=float("-inf") if self.kind == "max" else 0.0)
            pad = (0, 0)
        return pool1d_nwc(x, self.kind, self.pool_length, self.stride, pad).to(x.dtype)


class MaxPooling1D(_Pool1D):
    kind = "max"


class AveragePooling1D(_Pool1D):
    kind = "avg"


class _Pool3D(Layer):
    kind = "max"

    def __init__(self, pool_size=(2, 2, 2), strides=None, border_mode="valid", dim_ordering="th",
                 input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.pool_size = tuple(pool_size)
        self.strides = tuple(strides) if strides is not None else self.pool_size
        self.border_mode, self.dim_ordering = border_mode, dim_ordering

    def compute_output_shape(self, s):
        sp = s[2:5] if self.dim_ordering == "th" else s[1:4]
        o = tuple(_pool_out(d, k, st, self.border_mode) for d, k, st in zip(sp, self.pool_size, self.strides))
        return (None, s[1]) + o if self.dim_ordering == "th" else (None,) + o + (s[4],)

    def call(self, x):
        from zoo.ops.layers import pool3d_ndhwc
        xn = x if self.dim_ordering == "tf" else x.permute(0, 2, 3, 4, 1)
        if x.is_cuda:
            xn = xn.contiguous()
        y = pool3d_ndhwc(xn, self.kind, self.pool_size, self.strides).to(x.dtype)
        return y if self.dim_ordering == "tf" else y.permute(0, 4, 1, 2, 3)


class MaxPooling3D(_Pool3D):
    kind = "max"


class AveragePooling3D(_Pool3D):
    kind = "avg"


class GlobalAveragePooling1D(Layer):
    def compute_output_shape(self, s):
        return (None, s[2])

    def call(self, x):
        return x.mean(dim=1)


class GlobalMaxPooling1D(Layer):
    def compute_output_shape(self, s):
        return (None, s[2])

    def call(self, x):
        return x.max(dim=1).values


class GlobalAveragePooling2D(Layer):
    def __init__(self, dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim_ordering = dim_ordering

    def compute_output_shape(self, s):
        return (None, s[1] if self.dim_ordering == "th" else s[3])

    def call(self, x):
        if x.is_cuda and x.dim() == 4:
            xn = x.permute(0, 2, 3, 1) if self.dim_ordering == "th" else x
            c = xn.shape[-1]
            xp = xn if c % 8 == 0 else F.pad(xn, (0, (-c) % 8))
            return ops.global_avg_pool_nhwc(xp.contiguous()).to(x.dtype)[:, :c]
        return x.mean(dim=(2, 3)) if self.dim_ordering == "th" else x.mean(dim=(1, 2))


class GlobalMaxPooling2D(Layer):
    def __init__(self, dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim_ordering = dim_ordering

    def compute_output_shape(self, s):
        return (None, s[1] if self.dim_ordering == "th" else s[3])

    def call(self, x):
        return x.amax(dim=(2, 3)) if self.dim_ordering == "th" else x.amax(dim=(1, 2))


class GlobalAveragePooling3D(Layer):
    def __init__(self, dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.dim_ordering = dim_ordering

    def compute_output_shape(self, s):
        return (None, s[1] if self.dim_ordering == "th" else s[4])

    def call(self, x):
        return x.mean(dim=(2, 3, 4)) if self.dim_ordering == "th" else x.mean(dim=(1, 2, 3))


class GlobalMaxPooling3D(GlobalAveragePooling3D):
    def call(self, x):
        return x.amax(dim=(2, 3, 4)) if self.dim_ordering == "th" else x.amax(dim=(1, 2, 3))
