"""Normalization layers: BatchNormalization (BatchNormalization.scala:85-110),
LayerNorm (+InternalLayerNorm), LRN2D, WithinChannelLRN2D.

Channels-last 4-D (and 2-D) BatchNormalization with 8-aligned channels runs
on the native NHWC BN kernels; LayerNorm runs on the native row kernel.
BigDL momentum semantics: running = (1 - momentum) * running + momentum * batch.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.parallel.sync_bn import sync_batch_norm, sync_bn_active
from zoo.pipeline.api.keras.base import Layer, init_tensor



class BatchNormalization(Layer):
    def __init__(self, epsilon=0.001, mode=0, axis=1, momentum=0.99, beta_init="zero", gamma_init="one",
                 dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.epsilon, self.momentum = float(epsilon), float(momentum)
        self.beta_init, self.gamma_init, self.dim_ordering = beta_init, gamma_init, dim_ordering

    def build(self, input_shape):
        if len(input_shape) == 4:
            c = input_shape[1] if self.dim_ordering == "th" else input_shape[3]
        else:
            c = input_shape[-1]
        self.nc = c
        self.gamma = nn.Parameter(init_tensor(torch.empty(c), self.gamma_init, fan_in=c, fan_out=c))
        self.beta = nn.Parameter(init_tensor(torch.empty(c), self.beta_init, fan_in=c, fan_out=c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))

    def call(self, x):
        channels_last = x.dim() == 2 or (x.dim() == 4 and self.dim_ordering == "tf") or x.dim() == 3
        if self.training and sync_bn_active():  # SyncBN across data-parallel ranks (P5)
            cdim = -1 if channels_last else 1
            return sync_batch_norm(x, self.gamma, self.beta, self.running_mean, self.running_var, self.epsilon,
                                   self.momentum, channel_dim=cdim)
        if channels_last and x.is_cuda and self.nc % 8 == 0:
            y = ops.batch_norm_nhwc(x, self.gamma, self.beta, self.running_mean, self.running_var, self.epsilon,
                                    self.momentum, relu=False, training=self.training)
            return y.to(x.dtype)
        if x.dim() == 4 and x.is_cuda and self.nc % 8 == 0:
            # th ordering on the native NHWC kernel (a free view for channels-last memory)
            y = ops.batch_norm_nhwc(x.permute(0, 2, 3, 1).contiguous(), self.gamma, self.beta, self.running_mean,
                                    self.running_var, self.epsilon, self.momentum, relu=False,
                                    training=self.training)
            return y.to(x.dtype).permute(0, 3, 1, 2)
        if x.is_cuda and x.dim() == 4 and self.nc % 8:
            return self._padded_native(x, channels_last)
        if x.dim() == 4 and self.dim_ordering == "tf":
            xc = x.permute(0, 3, 1, 2)
        elif x.dim() == 3:
            xc = x.transpose(1, 2)
        else:
            xc = x
        # generic fallback (channel counts the NHWC kernel does not take) on ATen's own kernels,
        # not MIOpen's
        with torch.backends.cudnn.flags(enabled=False):
            y = F.batch_norm(xc, self.running_mean, self.running_var, self.gamma.to(xc.dtype),
                             self.beta.to(xc.dtype), self.training, self.momentum, self.epsilon)
        if x.dim() == 4 and self.dim_ordering == "tf":
            y = y.permute(0, 2, 3, 1)
        elif x.dim() == 3:
            y = y.transpose(1, 2)
        return y

    def _padded_native(self, x, channels_last):
        """Channel count off the kernel's 8-channel granule: zero-pad the channels (the pad
        channels normalise to beta = 0), run the native NHWC BN, slice, and write the updated
        running statistics back (was an ATen fallback)."""
        nc, cp = self.nc, (-self.nc) % 8
        xn = x if channels_last else x.permute(0, 2, 3, 1)
        xp = F.pad(xn, (0, cp)).contiguous()
        g = F.pad(self.gamma, (0, cp), value=1.0)
        b = F.pad(self.beta, (0, cp))
        rm = F.pad(self.running_mean, (0, cp)).contiguous()
        rv = F.pad(self.running_var, (0, cp), value=1.0).contiguous()
        y = ops.batch_norm_nhwc(xp, g, b, rm, rv, self.epsilon, self.momentum, relu=False, training=self.training)
        if self.training:
            with torch.no_grad():
                self.running_mean.copy_(rm[:nc])
                self.running_var.copy_(rv[:nc])
        y = y[..., :nc].to(x.dtype)
        return y if channels_last else y.permute(0, 3, 1, 2)

    def get_weights(self):
        return [self.gamma.detach().cpu().numpy().copy(), self.beta.detach().cpu().numpy().copy(),
                self.running_mean.cpu().numpy().copy(), self.running_var.cpu().numpy().copy()]

    def set_weights(self, weights):
        with torch.no_grad():
            self.gamma.copy_(torch.as_tensor(np.asarray(weights[0])))
            self.beta.copy_(torch.as_tensor(np.asarray(weights[1])))
            if len(weights) > 2:
                self.running_mean.copy_(torch.as_tensor(np.asarray(weights[2])))
                self.running_var.copy_(torch.as_tensor(np.asarray(weights[3])))


class LayerNorm(Layer):
    """y = (x - mean) / sqrt(var + eps) * weight + bias over the last dim (LayerNorm.scala)."""

    def __init__(self, n_output=768, epsilon=1e-5, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.n_output, self.epsilon = int(n_output), float(epsilon)

    def build(self, input_shape):
        self.weight = nn.Parameter(torch.ones(self.n_output))
        self.bias = nn.Parameter(torch.zeros(self.n_output))

    def call(self, x):
        return ops.layer_norm(x, self.weight, self.bias, self.epsilon)


class LRN2D(Layer):
    """Cross-channel local response normalization (SpatialCrossMapLRN)."""

    def __init__(self, alpha=1e-4, k=1.0, beta=0.75, n=5, dim_ordering="th", input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.alpha, self.k, self.beta, self.n, self.dim_ordering = alpha, k, beta, n, dim_ordering

    def call(self, x):
        # y = x / (k + alpha * sum_{n channels} x^2)^beta (Keras-1 LRN2D) on the native
        # channels-last LRN kernel (its window scale is alpha / n)
        xn = x.permute(0, 2, 3, 1) if self.dim_ordering == "th" else x
        y = ops.lrn_channels_last(xn.contiguous(), self.n, self.alpha * self.n, self.beta, self.k)
        return y.permute(0, 3, 1, 2) if self.dim_ordering == "th" else y


class WithinChannelLRN2D(Layer):
    """Normalization over a spatial size x size window inside each channel."""

    def __init__(self, size=5, alpha=1.0, beta=0.75, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.size, self.alpha, self.beta = int(size), float(alpha), float(beta)

    def call(self, x):
        # SpatialWithinChannelLRN ('th' input): native NHWC kernel (size x size window mean of x^2)
        from zoo.ops.layers import within_channel_lrn
        y = within_channel_lrn(x.permute(0, 2, 3, 1).contiguous(), self.size, self.alpha, self.beta)
        return y.permute(0, 3, 1, 2)
