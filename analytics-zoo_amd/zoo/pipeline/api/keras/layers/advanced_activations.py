"""Advanced activations and elementwise layers (advanced_activations.py,
noise.py and the BigDL-module wrappers of torch.py in the reference:
LeakyReLU, ELU, ThresholdedReLU, SReLU, PReLU, RReLU, HardTanh, HardShrink,
SoftShrink, Threshold, BinaryThreshold, AddConstant, MulConstant, CAdd, CMul,
Exp, Log, Power, Sqrt, Square, Negative, Scale, Mul, Identity,
GaussianNoise, GaussianDropout, GaussianSampler)."""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo.pipeline.api.keras.base import Layer, init_tensor, to_shape


class LeakyReLU(Layer):
    def __init__(self, alpha=0.01, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.alpha = float(alpha)

    def call(self, x):
        return F.leaky_relu(x, self.alpha)


class ELU(Layer):
    def __init__(self, alpha=1.0, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.alpha = float(alpha)

    def call(self, x):
        return F.elu(x, self.alpha)


class ThresholdedReLU(Layer):
    def __init__(self, theta=1.0, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.theta = float(theta)

    def call(self, x):
        return x * (x > self.theta).to(x.dtype)


class SReLU(Layer):
    """S-shaped ReLU with learnable (t_left, a_left, t_right, a_right) per feature."""

    def __init__(self, t_left_init="zero", a_left_init="glorot_uniform", t_right_init="glorot_uniform",
                 a_right_init="one", shared_axes=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.inits = (t_left_init, a_left_init, t_right_init, a_right_init)
        self.shared_axes = shared_axes

    def build(self, input_shape):
        shape = list(input_shape[1:])
        if self.shared_axes:
            for a in self.shared_axes:
                shape[a - 1] = 1
        shape = tuple(shape)
        n = int(np.prod(shape))
        for name, init in zip(("t_left", "a_left", "t_right", "a_right"), self.inits):
            setattr(self, name, nn.Parameter(init_tensor(torch.empty(shape), init, fan_in=n, fan_out=n)))

    def call(self, x):
        tr = self.t_left + self.t_right.abs()
        y = torch.where(x >= tr, tr + self.a_right * (x - tr), x)
        return torch.where(x <= self.t_left, self.t_left + self.a_left * (x - self.t_left), y)


class PReLU(Layer):
    def __init__(self, n_output_plane=0, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.n = int(n_output_plane)

    def build(self, input_shape):
        self.weight = nn.Parameter(torch.full((max(self.n, 1),), 0.25))

    def call(self, x):
        w = self.weight
        if self.n > 0 and x.dim() > 2:
            shape = [1, self.n] + [1] * (x.dim() - 2)
            w = w.reshape(shape)
        return torch.where(x >= 0, x, w.to(x.dtype) * x)


class RReLU(Layer):
    def __init__(self, lower=1.0 / 8, upper=1.0 / 3, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.lower, self.upper = float(lower), float(upper)

    def call(self, x):
        return F.rrelu(x, self.lower, self.upper, self.training)


class HardTanh(Layer):
    def __init__(self, min_value=-1, max_value=1, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.lo, self.hi = float(min_value), float(max_value)

    def call(self, x):
        return torch.clamp(x, self.lo, self.hi)


class HardShrink(Layer):
    def __init__(self, value=0.5, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.value = float(value)

    def call(self, x):
        return F.hardshrink(x, self.value)


class SoftShrink(Layer):
    def __init__(self, value=0.5, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.value = float(value)

    def call(self, x):
        return F.softshrink(x, self.value)


class Threshold(Layer):
    def __init__(self, th=1e-6, v=0.0, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.th, self.v = float(th), float(v)

    def call(self, x):
        return torch.where(x > self.th, x, torch.full_like(x, self.v))


class BinaryThreshold(Layer):
    def __init__(self, value=1e-6, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.value = float(value)

    def call(self, x):
        return (x > self.value).to(x.dtype)


class AddConstant(Layer):
    def __init__(self, constant, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.constant = float(constant)

    def call(self, x):
        return x + self.constant


class MulConstant(Layer):
    def __init__(self, constant, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.constant = float(constant)

    def call(self, x):
        return x * self.constant


class CAdd(Layer):
    """Learnable broadcast bias of ``size`` (excl. batch)."""

    def __init__(self, size, b_regularizer=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.size = to_shape(size)
        self.add_regularizer(b_regularizer, "bias")

    def build(self, input_shape):
        self.bias = nn.Parameter(torch.zeros(self.size))

    def call(self, x):
        return x + self.bias.to(x.dtype)


class CMul(Layer):
    def __init__(self, size, W_regularizer=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.size = to_shape(size)
        self.add_regularizer(W_regularizer, "weight")

    def build(self, input_shape):
        self.weight = nn.Parameter(torch.ones(self.size))

    def call(self, x):
        return x * self.weight.to(x.dtype)


class Scale(Layer):
    """CMul then CAdd with parameters of ``size``."""

    def __init__(self, size, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.size = to_shape(size)

    def build(self, input_shape):
        self.weight = nn.Parameter(torch.ones(self.size))
        self.bias = nn.Parameter(torch.zeros(self.size))

    def call(self, x):
        return x * self.weight.to(x.dtype) + self.bias.to(x.dtype)


class Mul(Layer):
    """Multiply by one learnable scalar."""

    def build(self, input_shape):
        self.weight = nn.Parameter(torch.ones(1))

    def call(self, x):
        return x * self.weight.to(x.dtype)


class Exp(Layer):
    def call(self, x):
        return torch.exp(x)


class Log(Layer):
    def call(self, x):
        return torch.log(x)


class Sqrt(Layer):
    def call(self, x):
        return torch.sqrt(x)


class Square(Layer):
    def call(self, x):
        return x * x


class Negative(Layer):
    def call(self, x):
        return -x


class Identity(Layer):
    def call(self, x):
        return x


class Power(Layer):
    """(shift + scale * x) ^ power"""

    def __init__(self, power, scale=1, shift=0, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.power, self.scale, self.shift = float(power), float(scale), float(shift)

    def call(self, x):
        return torch.pow(self.shift + self.scale * x, self.power)


class GaussianNoise(Layer):
    def __init__(self, sigma, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.sigma = float(sigma)

    def call(self, x):
        return x + torch.randn_like(x) * self.sigma if self.training else x


class GaussianDropout(Layer):
    def __init__(self, p, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.p = float(p)

    def call(self, x):
        if not self.training or self.p == 0:
            return x
        std = (self.p / (1 - self.p)) ** 0.5
        return x * (1 + torch.randn_like(x) * std)


class GaussianSampler(Layer):
    """Takes [mean, log_variance] and samples mean + exp(logvar/2) * eps (VAE)."""

    def compute_output_shape(self, input_shape):
        return input_shape[0]

    def call(self, x):
        mu, logvar = x
        return mu + torch.exp(0.5 * logvar) * torch.randn_like(mu)
