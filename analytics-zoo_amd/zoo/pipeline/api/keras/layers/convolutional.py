"""Convolution-family Keras layers.

Parity: Py/pipeline/api/keras/layers/convolutional.py and the Scala layers
Convolution1D/2D/3D, AtrousConvolution1D/2D, Deconvolution2D,
SeparableConvolution2D, ShareConvolution2D, LocallyConnected1D/2D,
UpSampling1D/2D/3D, ZeroPadding1D/2D/3D, Cropping1D/2D/3D, ResizeBilinear.

2-D / 1-D convolutions (incl. atrous and transposed) run on the native
implicit-GEMM MFMA kernels in NHWC. ``dim_ordering="tf"`` (channels last) is
the zero-copy fast path; ``"th"`` (channels first, the Keras-1 default) is
supported by transposing at the layer boundary. Channel counts that are not
8-aligned are zero-padded internally (weights and activations) so every
conv stays on the MFMA path. 3-D, depthwise and locally-connected
convolutions use PyTorch-ROCm kernels.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.ops import layers as ops_layers
from zoo.pipeline.api.keras.base import Layer, apply_activation, check_activation, init_tensor, to_shape


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)


def _native_cin(c):
    return c if c % 8 == 0 else (4 if c <= 4 else ops.ceil8(c))


def _same_pads(size, k, stride, dil=1):
    eff = dil * (k - 1) + 1
    out = int(math.ceil(size / stride))
    total = max((out - 1) * stride + eff - size, 0)
    return total // 2, total - total // 2


class _Conv2DBase(Layer):
    """Shared NHWC conv machinery with packed weights."""

    def _setup(self, nb_filter, kernel, init, activation, border_mode, subsample, dim_ordering, dilation,
               W_regularizer, b_regularizer, bias):
        self.nb_filter = int(nb_filter)
        self.kernel = _pair(kernel)
        self.init = init
        self.activation = check_activation(activation)
        self.border_mode = border_mode
        self.subsample = _pair(subsample)
        self.dim_ordering = dim_ordering
        self.dilation = _pair(dilation)
        self.use_bias = bias
        self.add_regularizer(W_regularizer, "weight")
        self.add_regularizer(b_regularizer, "bias")

    def _in_channels(self, shape):
        return shape[1] if self.dim_ordering == "th" else shape[-1]

    def build(self, input_shape):
        c = self._in_channels(input_shape)
        self.cin = c
        self.cin_p = _native_cin(c)
        self.k_p = ops.ceil8(self.nb_filter)
        R, S = self.kernel
        w4 = torch.zeros(self.k_p, R, S, self.cin_p)
        logical = torch.empty(self.nb_filter, c, R, S)
        init_tensor(logical, self.init)
        w4[: self.nb_filter, :, :, :c] = logical.permute(0, 2, 3, 1)
        self.weight = nn.Parameter(ops.pack_weight(w4))
        self.bias = nn.Parameter(torch.zeros(self.k_p)) if self.use_bias else None

    def _spatial(self, shape):
        return (shape[2], shape[3]) if self.dim_ordering == "th" else (shape[1], shape[2])

    def _pads(self, hw):
        if self.border_mode == "same":
            return [_same_pads(hw[i], self.kernel[i], self.subsample[i], self.dilation[i]) for i in range(2)]
        if isinstance(self.border_mode, (tuple, list)):
            p = _pair(self.border_mode)
            return [(p[0], p[0]), (p[1], p[1])]
        return [(0, 0), (0, 0)]

    def compute_output_shape(self, input_shape):
        hw = self._spatial(input_shape)
        pads = self._pads(hw)
        out = []
        for i in range(2):
            if hw[i] is None:
                out.append(None)
                continue
            out.append((hw[i] + pads[i][0] + pads[i][1] - self.dilation[i] * (self.kernel[i] - 1) - 1)
                       // self.subsample[i] + 1)
        if self.dim_ordering == "th":
            return (None, self.nb_filter, out[0], out[1])
        return (None, out[0], out[1], self.nb_filter)

    def _conv_nhwc(self, x):
        """x: NHWC (any float dtype) -> NHWC with nb_filter channels."""
        pads = self._pads((x.shape[1], x.shape[2]))
        sym = [pads[0][0], pads[1][0]]
        extra = (pads[0][1] - pads[0][0], pads[1][1] - pads[1][0])
        if extra[0] or extra[1] or self.cin_p != x.shape[-1]:
            x = F.pad(x, (0, self.cin_p - x.shape[-1], 0, extra[1], 0, extra[0]))
        act = self.activation.lower() if isinstance(self.activation, str) else self.activation
        fuse = act in (None, "linear", "relu", "sigmoid", "tanh")
        y = ops.conv2d_nhwc(x, self.weight, self.bias, kernel=self.kernel, stride=self.subsample, pad=sym,
                            dil=self.dilation, act=act if fuse else None, out_f32=x.dtype == torch.float32)
        if self.k_p != self.nb_filter:
            y = y[..., : self.nb_filter]
        if not fuse:
            y = apply_activation(y, self.activation)
        return y

    def call(self, x):
        if self.dim_ordering == "th":
            # channels-last propagation: the NCHW result is a view of the NHWC output
            # (torch.channels_last memory), so the next th layer's permute back to NHWC is
            # free; only the graph input pays one NCHW -> NHWC copy
            y = self._conv_nhwc(x.permute(0, 2, 3, 1))
            return y.permute(0, 3, 1, 2)
        return self._conv_nhwc(x).contiguous()

    # ---- weights in the reference layouts ----
    def _logical(self):
        R, S = self.kernel
        w = ops.unpack_weight(self.weight.detach().float().cpu(), self.k_p, R, S, self.cin_p)
        return w[: self.nb_filter, :, :, : self.cin]  # [K][R][S][C]

    def get_weights(self):
        w = self._logical()
        w = w.permute(0, 3, 1, 2) if self.dim_ordering == "th" else w.permute(1, 2, 3, 0)
        out = [w.numpy().copy()]
        if self.bias is not None:
            out.append(self.bias.detach().float().cpu()[: self.nb_filter].numpy().copy())
        return out

    def set_weights(self, weights):
        R, S = self.kernel
        w = torch.as_tensor(np.asarray(weights[0]), dtype=torch.float32)
        w = w.reshape(self.nb_filter, self.cin, R, S).permute(0, 2, 3, 1) if self.dim_ordering == "th" else \
            w.reshape(R, S, self.cin, self.nb_filter).permute(3, 0, 1, 2)
        w4 = torch.zeros(self.k_p, R, S, self.cin_p)
        w4[: self.nb_filter, :, :, : self.cin] = w
        with torch.no_grad():
            self.weight.copy_(ops.pack_weight(w4).to(self.weight.device))
            if self.bias is not None and len(weights) > 1:
                self.bias.zero_()
                self.bias[: self.nb_filter].copy_(torch.as_tensor(np.asarray(weights[1])))


class Convolution2D(_Conv2DBase):
    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample=(1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None, bias=True,
                 input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self._setup(nb_filter, (nb_row, nb_col), init, activation, border_mode, subsample, dim_ordering, (1, 1),
                    W_regularizer, b_regularizer, bias)


Conv2D = Convolution2D


class ShareConvolution2D(Convolution2D):
    """Weight-shared conv (ShareConvolution2D.scala); identical math here."""

    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, subsample=(1, 1),
                 pad_h=0, pad_w=0, propagate_back=True, dim_ordering="th", W_regularizer=None, b_regularizer=None,
                 bias=True, input_shape=None, **kwargs):
        super().__init__(nb_filter, nb_row, nb_col, init, activation, (pad_h, pad_w), subsample, dim_ordering,
                         W_regularizer, b_regularizer, bias, input_shape, **kwargs)


class AtrousConvolution2D(_Conv2DBase):
    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample=(1, 1), atrous_rate=(1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None,
                 bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self._setup(nb_filter, (nb_row, nb_col), init, activation, border_mode, subsample, dim_ordering,
                    atrous_rate, W_regularizer, b_regularizer, bias)


class Convolution1D(_Conv2DBase):
    """Temporal conv over (batch, steps, input_dim) — an NHWC conv with H = 1."""

    def __init__(self, nb_filter, filter_length, init="glorot_uniform", limits=None, activation=None,
                 border_mode="valid", subsample_length=1, W_regularizer=None, b_regularizer=None, bias=True,
                 input_shape=None, dilation=1, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self._setup(nb_filter, (1, filter_length), init, activation, border_mode, (1, subsample_length), "tf",
                    (1, dilation), W_regularizer, b_regularizer, bias)

    def _in_channels(self, shape):
        return shape[-1]

    def compute_output_shape(self, input_shape):
        s = super().compute_output_shape((None, 1, input_shape[1], input_shape[2]))
        return (None, s[2], s[3])

    def _pads(self, hw):
        p = super()._pads(hw)
        return [(0, 0), p[1]]

    def call(self, x):
        return self._conv_nhwc(x.unsqueeze(1)).squeeze(1)

    def get_weights(self):
        w = self._logical()[:, 0]  # [K][S][C]
        out = [w.permute(1, 2, 0).numpy().copy()]
        if self.bias is not None:
            out.append(self.bias.detach().float().cpu()[: self.nb_filter].numpy().copy())
        return out

    def set_weights(self, weights):
        w = torch.as_tensor(np.asarray(weights[0]), dtype=torch.float32)  # [S][C][K]
        S = self.kernel[1]
        w = w.reshape(S, self.cin, self.nb_filter).permute(2, 0, 1).unsqueeze(1)  # [K][1][S][C]
        w4 = torch.zeros(self.k_p, 1, S, self.cin_p)
        w4[: self.nb_filter, :, :, : self.cin] = w
        with torch.no_grad():
            self.weight.copy_(ops.pack_weight(w4).to(self.weight.device))
            if self.bias is not None and len(weights) > 1:
                self.bias.zero_()
                self.bias[: self.nb_filter].copy_(torch.as_tensor(np.asarray(weights[1])))


Conv1D = Convolution1D


class AtrousConvolution1D(Convolution1D):
    def __init__(self, nb_filter, filter_length, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample_length=1, atrous_rate=1, W_regularizer=None, b_regularizer=None, bias=True,
                 input_shape=None, **kwargs):
        super().__init__(nb_filter, filter_length, init, None, activation, border_mode, subsample_length,
                         W_regularizer, b_regularizer, bias, input_shape, dilation=atrous_rate, **kwargs)


class Deconvolution2D(Layer):
    """Transposed convolution on the native dgrad kernel path (SpatialFullConvolution)."""

    def __init__(self, nb_filter, nb_row, nb_col, output_shape=None, init="glorot_uniform", activation=None,
                 border_mode="valid", subsample=(1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None,
                 bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.kernel, self.subsample = int(nb_filter), (nb_row, nb_col), _pair(subsample)
        self.init, self.activation, self.dim_ordering, self.use_bias = init, activation, dim_ordering, bias
        self.given_output_shape = output_shape

    def build(self, input_shape):
        c = input_shape[1] if self.dim_ordering == "th" else input_shape[-1]
        self.cin, self.cin_p, self.k_p = c, ops.ceil8(c), ops.ceil8(self.nb_filter)
        R, S = self.kernel
        wd = init_tensor(torch.empty(c, self.nb_filter, R, S), self.init)  # BigDL [in][out][kh][kw]
        wf = torch.zeros(self.cin_p, R, S, self.k_p)
        wf[:c, :, :, : self.nb_filter] = wd.permute(0, 2, 3, 1)
        self.weight = nn.Parameter(ops.pack_weight(wf))
        self.bias = nn.Parameter(torch.zeros(self.nb_filter)) if self.use_bias else None

    def _out_hw(self, h, w):
        return ((h - 1) * self.subsample[0] + self.kernel[0], (w - 1) * self.subsample[1] + self.kernel[1])

    def compute_output_shape(self, input_shape):
        if self.dim_ordering == "th":
            oh, ow = self._out_hw(input_shape[2], input_shape[3])
            return (None, self.nb_filter, oh, ow)
        oh, ow = self._out_hw(input_shape[1], input_shape[2])
        return (None, oh, ow, self.nb_filter)

    def call(self, x):
        xh = x.permute(0, 2, 3, 1) if self.dim_ordering == "th" else x
        if xh.shape[-1] != self.cin_p:
            xh = F.pad(xh, (0, self.cin_p - xh.shape[-1]))
        oh, ow = self._out_hw(xh.shape[1], xh.shape[2])
        y = ops.conv.conv_transpose2d_nhwc(xh, self.weight, self.kernel, self.subsample, (0, 0), (oh, ow), self.k_p)
        y = y[..., : self.nb_filter]
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        y = apply_activation(y, self.activation)
        if x.dtype == torch.float32:
            y = y.float()
        return y.permute(0, 3, 1, 2).contiguous() if self.dim_ordering == "th" else y.contiguous()


class SeparableConvolution2D(Layer):
    """Depthwise (PyTorch grouped conv) followed by a native 1x1 pointwise conv."""

    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample=(1, 1), depth_multiplier=1, dim_ordering="th", depthwise_regularizer=None,
                 pointwise_regularizer=None, b_regularizer=None, bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.kernel, self.subsample = int(nb_filter), (nb_row, nb_col), _pair(subsample)
        self.init, self.activation, self.border_mode = init, activation, border_mode
        self.depth_multiplier, self.dim_ordering, self.use_bias = int(depth_multiplier), dim_ordering, bias

    def build(self, input_shape):
        c = input_shape[1] if self.dim_ordering == "th" else input_shape[-1]
        self.cin = c
        R, S = self.kernel
        self.depthwise = nn.Parameter(init_tensor(torch.empty(c * self.depth_multiplier, 1, R, S), self.init))
        self.pointwise = nn.Parameter(init_tensor(torch.empty(self.nb_filter, c * self.depth_multiplier), self.init))
        self.bias = nn.Parameter(torch.zeros(self.nb_filter)) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        hw = (input_shape[2], input_shape[3]) if self.dim_ordering == "th" else (input_shape[1], input_shape[2])
        out = []
        for i in range(2):
            if self.border_mode == "same":
                out.append(int(math.ceil(hw[i] / self.subsample[i])))
            else:
                out.append((hw[i] - self.kernel[i]) // self.subsample[i] + 1)
        return (None, self.nb_filter, out[0], out[1]) if self.dim_ordering == "th" else \
            (None, out[0], out[1], self.nb_filter)

    def call(self, x):
        if x.is_cuda and self.kernel[0] * self.kernel[1] <= 9 and (self.cin * self.depth_multiplier) % 8 == 0:
            # native: depthwise kernel (NHWC) -> pointwise 1x1 on the implicit-GEMM conv
            xn = x.permute(0, 2, 3, 1) if self.dim_ordering == "th" else x
            if self.border_mode == "same":
                p = [_same_pads(xn.shape[1 + i], self.kernel[i], self.subsample[i]) for i in range(2)]
                xn = F.pad(xn, (0, 0, p[1][0], p[1][1], p[0][0], p[0][1]))
            if self.depth_multiplier > 1:
                xn = xn.repeat_interleave(self.depth_multiplier, dim=-1)
            R, S = self.kernel
            taps = self.depthwise.reshape(self.cin * self.depth_multiplier, R * S).t()   # [R*S, C*m]
            d = ops.depthwise_conv2d_nhwc(xn, taps, None, kernel=(R, S), stride=self.subsample)
            y = ops.linear(d, self.pointwise, self.bias)
            y = apply_activation(y, self.activation).to(x.dtype)
            return y.permute(0, 3, 1, 2).contiguous() if self.dim_ordering == "th" else y
        xc = x if self.dim_ordering == "th" else x.permute(0, 3, 1, 2)
        pad = 0
        if self.border_mode == "same":
            p = [_same_pads(xc.shape[2 + i], self.kernel[i], self.subsample[i]) for i in range(2)]
            xc = F.pad(xc, (p[1][0], p[1][1], p[0][0], p[0][1]))
        d = F.conv2d(xc, self.depthwise.to(xc.dtype), stride=self.subsample, padding=pad, groups=self.cin)
        y = ops.linear(d.permute(0, 2, 3, 1), self.pointwise, self.bias)
        y = apply_activation(y, self.activation)
        return y.permute(0, 3, 1, 2).contiguous() if self.dim_ordering == "th" else y


class Convolution3D(Layer):
    def __init__(self, nb_filter, kernel_dim1, kernel_dim2, kernel_dim3, init="glorot_uniform", activation=None,
                 border_mode="valid", subsample=(1, 1, 1), dim_ordering="th", W_regularizer=None,
                 b_regularizer=None, bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.kernel = int(nb_filter), (kernel_dim1, kernel_dim2, kernel_dim3)
        self.init, self.activation, self.border_mode = init, activation, border_mode
        self.subsample, self.dim_ordering, self.use_bias = tuple(subsample), dim_ordering, bias
        self.add_regularizer(W_regularizer, "weight")

    def build(self, input_shape):
        c = input_shape[1] if self.dim_ordering == "th" else input_shape[-1]
        self.weight = nn.Parameter(init_tensor(torch.empty((self.nb_filter, c) + self.kernel), self.init))
        self.bias = nn.Parameter(torch.zeros(self.nb_filter)) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        sp = input_shape[2:5] if self.dim_ordering == "th" else input_shape[1:4]
        out = [int(math.ceil(s / st)) if self.border_mode == "same" else (s - k) // st + 1
               for s, k, st in zip(sp, self.kernel, self.subsample)]
        return (None, self.nb_filter, *out) if self.dim_ordering == "th" else (None, *out, self.nb_filter)

    def call(self, x):
        from zoo.ops.layers import conv3d_ndhwc
        xn = x if self.dim_ordering == "tf" else x.permute(0, 2, 3, 4, 1)        # NDHWC
        if self.border_mode == "same":
            p = [_same_pads(xn.shape[1 + i], self.kernel[i], self.subsample[i]) for i in range(3)]
            xn = F.pad(xn, (0, 0, p[2][0], p[2][1], p[1][0], p[1][1], p[0][0], p[0][1]))
        K, C = self.weight.shape[0], self.weight.shape[1]
        if x.is_cuda and (C % 8 or K % 8):   # 16-byte channel granule of the MFMA conv: zero-pad
            cp, kp = (-C) % 8, (-K) % 8
            xn = F.pad(xn, (0, cp))
            w5 = F.pad(self.weight.permute(0, 2, 3, 4, 1), (0, cp, 0, 0, 0, 0, 0, 0, 0, kp))
            b = None if self.bias is None else F.pad(self.bias, (0, kp))
            y = conv3d_ndhwc(xn.to(torch.bfloat16), w5, b, stride=self.subsample)[..., :K]
        else:
            y = conv3d_ndhwc(xn.to(torch.bfloat16) if x.is_cuda else xn, self.weight.permute(0, 2, 3, 4, 1),
                             self.bias, stride=self.subsample)
        y = apply_activation(y.to(x.dtype), self.activation)
        return y if self.dim_ordering == "tf" else y.permute(0, 4, 1, 2, 3)


Conv3D = Convolution3D


class LocallyConnected2D(Layer):
    """Unshared-weight 2-D conv via unfold + batched GEMM."""

    def __init__(self, nb_filter, nb_row, nb_col, activation=None, border_mode="valid", subsample=(1, 1),
                 dim_ordering="th", W_regularizer=None, b_regularizer=None, bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.kernel, self.subsample = int(nb_filter), (nb_row, nb_col), _pair(subsample)
        self.activation, self.dim_ordering, self.use_bias = activation, dim_ordering, bias

    def build(self, input_shape):
        c, h, w = (input_shape[1], input_shape[2], input_shape[3]) if self.dim_ordering == "th" else \
            (input_shape[3], input_shape[1], input_shape[2])
        self.oh = (h - self.kernel[0]) // self.subsample[0] + 1
        self.ow = (w - self.kernel[1]) // self.subsample[1] + 1
        L, Kd = self.oh * self.ow, c * self.kernel[0] * self.kernel[1]
        self.weight = nn.Parameter(init_tensor(torch.empty(L, Kd, self.nb_filter), "glorot_uniform",
                                               fan_in=Kd, fan_out=self.nb_filter))
        self.bias = nn.Parameter(torch.zeros(L, self.nb_filter)) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        return (None, self.nb_filter, self.oh, self.ow) if self.dim_ordering == "th" else \
            (None, self.oh, self.ow, self.nb_filter)

    def call(self, x):
        xc = x if self.dim_ordering == "th" else x.permute(0, 3, 1, 2)
        cols = F.unfold(xc, self.kernel, stride=self.subsample)          # [N, Kd, L]
        y = torch.einsum("nkl,lko->nlo", cols, self.weight.to(cols.dtype))
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        y = apply_activation(y, self.activation)                          # [N, L, O]
        y = y.reshape(x.shape[0], self.oh, self.ow, self.nb_filter)
        return y.permute(0, 3, 1, 2).contiguous() if self.dim_ordering == "th" else y


class LocallyConnected1D(Layer):
    def __init__(self, nb_filter, filter_length, activation=None, border_mode="valid", subsample_length=1,
                 W_regularizer=None, b_regularizer=None, bias=True, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.k, self.s, self.activation, self.use_bias = int(nb_filter), filter_length, \
            subsample_length, activation, bias

    def build(self, input_shape):
        steps, d = input_shape[1], input_shape[2]
        self.out_steps = (steps - self.k) // self.s + 1
        self.weight = nn.Parameter(init_tensor(torch.empty(self.out_steps, self.k * d, self.nb_filter),
                                               "glorot_uniform", fan_in=self.k * d, fan_out=self.nb_filter))
        self.bias = nn.Parameter(torch.zeros(self.out_steps, self.nb_filter)) if self.use_bias else None

    def compute_output_shape(self, input_shape):
        return (None, self.out_steps, self.nb_filter)

    def call(self, x):
        win = x.unfold(1, self.k, self.s)                                  # [N, L, D, k]
        win = win.permute(0, 1, 3, 2).reshape(x.shape[0], self.out_steps, -1)
        y = torch.einsum("nlk,lko->nlo", win, self.weight.to(win.dtype))
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return apply_activation(y, self.activation)


# ---------------------------------------------------------------------------
# resampling / padding / cropping
# ---------------------------------------------------------------------------
class UpSampling1D(Layer):
    def __init__(self, length=2, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.length = int(length)

    def compute_output_shape(self, s):
        return (None, None if s[1] is None else s[1] * self.length, s[2])

    def call(self, x):
        return ops_layers.upsample_nearest(x, (self.length,))


class UpSampling2D(Layer):
    def __init__(self, size=(2, 2), dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.size, self.dim_ordering = _pair(size), dim_ordering

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (None, s[1], s[2] * self.size[0], s[3] * self.size[1])
        return (None, s[1] * self.size[0], s[2] * self.size[1], s[3])

    def call(self, x):
        if self.dim_ordering == "th":
            return ops_layers.upsample_nearest(x.permute(0, 2, 3, 1), self.size).permute(0, 3, 1, 2)
        return ops_layers.upsample_nearest(x, self.size)


class UpSampling3D(Layer):
    def __init__(self, size=(2, 2, 2), dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.size, self.dim_ordering = tuple(size), dim_ordering

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (None, s[1]) + tuple(d * k for d, k in zip(s[2:], self.size))
        return (None,) + tuple(d * k for d, k in zip(s[1:4], self.size)) + (s[4],)

    def call(self, x):
        if self.dim_ordering == "th":
            return ops_layers.upsample_nearest(x.permute(0, 2, 3, 4, 1), self.size).permute(0, 4, 1, 2, 3)
        return ops_layers.upsample_nearest(x, self.size)


class ZeroPadding1D(Layer):
    def __init__(self, padding=1, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.padding = _pair(padding)

    def compute_output_shape(self, s):
        return (None, s[1] + sum(self.padding), s[2])

    def call(self, x):
        return F.pad(x, (0, 0, self.padding[0], self.padding[1]))


class ZeroPadding2D(Layer):
    def __init__(self, padding=(1, 1), dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        p = tuple(padding)
        self.pad = (p[0], p[0], p[1], p[1]) if len(p) == 2 else p
        self.dim_ordering = dim_ordering

    def compute_output_shape(self, s):
        t, b, l, r = self.pad
        if self.dim_ordering == "th":
            return (None, s[1], s[2] + t + b, s[3] + l + r)
        return (None, s[1] + t + b, s[2] + l + r, s[3])

    def call(self, x):
        t, b, l, r = self.pad
        if self.dim_ordering == "th":
            return F.pad(x, (l, r, t, b))
        return F.pad(x, (0, 0, l, r, t, b))


class ZeroPadding3D(Layer):
    def __init__(self, padding=(1, 1, 1), dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.padding, self.dim_ordering = tuple(padding), dim_ordering

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (None, s[1]) + tuple(d + 2 * p for d, p in zip(s[2:], self.padding))
        return (None,) + tuple(d + 2 * p for d, p in zip(s[1:4], self.padding)) + (s[4],)

    def call(self, x):
        a, b, c = self.padding
        if self.dim_ordering == "th":
            return F.pad(x, (c, c, b, b, a, a))
        return F.pad(x, (0, 0, c, c, b, b, a, a))


class Cropping1D(Layer):
    def __init__(self, cropping=(1, 1), input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.cropping = tuple(cropping)

    def compute_output_shape(self, s):
        return (None, s[1] - sum(self.cropping), s[2])

    def call(self, x):
        return x[:, self.cropping[0]: x.shape[1] - self.cropping[1]]


class Cropping2D(Layer):
    def __init__(self, cropping=((0, 0), (0, 0)), dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.cropping, self.dim_ordering = tuple(tuple(c) for c in cropping), dim_ordering

    def compute_output_shape(self, s):
        (t, b), (l, r) = self.cropping
        if self.dim_ordering == "th":
            return (None, s[1], s[2] - t - b, s[3] - l - r)
        return (None, s[1] - t - b, s[2] - l - r, s[3])

    def call(self, x):
        (t, b), (l, r) = self.cropping
        if self.dim_ordering == "th":
            return x[:, :, t: x.shape[2] - b, l: x.shape[3] - r]
        return x[:, t: x.shape[1] - b, l: x.shape[2] - r]


class Cropping3D(Layer):
    def __init__(self, cropping=((1, 1), (1, 1), (1, 1)), dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.cropping, self.dim_ordering = tuple(tuple(c) for c in cropping), dim_ordering

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (None, s[1]) + tuple(d - a - b for d, (a, b) in zip(s[2:], self.cropping))
        return (None,) + tuple(d - a - b for d, (a, b) in zip(s[1:4], self.cropping)) + (s[4],)

    def call(self, x):
        o = 2 if self.dim_ordering == "th" else 1
        idx = [slice(None)] * x.dim()
        for i, (a, b) in enumerate(self.cropping):
            idx[o + i] = slice(a, x.shape[o + i] - b)
        return x[tuple(idx)]


class ResizeBilinear(Layer):
    def __init__(self, output_height, output_width, align_corner=False, dim_ordering="th", input_shape=None,
                 **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.oh, self.ow, self.align, self.dim_ordering = output_height, output_width, align_corner, dim_ordering

    def compute_output_shape(self, s):
        return (None, s[1], self.oh, self.ow) if self.dim_ordering == "th" else (None, self.oh, self.ow, s[3])

    def call(self, x):
        # BigDL nn.ResizeBilinear sampling (TF legacy: src = dst * in/out, or (in-1)/(out-1)
        # with align_corners); native NHWC kernel on the GPU
        xn = x.permute(0, 2, 3, 1) if self.dim_ordering == "th" else x
        y = ops_layers.resize_bilinear(xn.contiguous(), self.oh, self.ow, self.align)
        return y.permute(0, 3, 1, 2) if self.dim_ordering == "th" else y
