"""Keras-2 style layer API (Zs/pipeline/api/keras2/layers/*.scala, Py/pipeline/api/keras2/layers/).

Keras-2 argument names (units, filters, kernel_size, strides, padding,
data_format, kernel_initializer, use_bias, ...) mapped onto the framework's
Keras-1 layers, so both APIs share one implementation (native NHWC conv /
MFMA dense kernels) and one serialization format.
"""
from zoo.pipeline.api.keras import layers as K1
from zoo.pipeline.api.keras.engine.topology import Merge


def _fmt(data_format):
    return "tf" if data_format in (None, "channels_last") else "th"


def _reg(r):
    return r


class Dense(K1.Dense):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zero", kernel_regularizer=None, bias_regularizer=None, input_dim=None,
                 input_shape=None, **kwargs):
        super().__init__(units, init=kernel_initializer, activation=activation, W_regularizer=kernel_regularizer,
                         b_regularizer=bias_regularizer, bias=use_bias, input_dim=input_dim, input_shape=input_shape,
                         **kwargs)


class Activation(K1.Activation):
    pass


class Dropout(K1.Dropout):
    def __init__(self, rate, noise_shape=None, seed=None, input_shape=None, **kwargs):
        super().__init__(rate, input_shape=input_shape, **kwargs)


class Flatten(K1.Flatten):
    def __init__(self, data_format=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)


class Softmax(K1.Activation):
    def __init__(self, axis=-1, input_shape=None, **kwargs):
        super().__init__("softmax", input_shape=input_shape, **kwargs)


class Conv1D(K1.Convolution1D):
    def __init__(self, filters, kernel_size, strides=1, padding="valid", dilation_rate=1, activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zero",
                 kernel_regularizer=None, bias_regularizer=None, input_shape=None, **kwargs):
        k = kernel_size[0] if isinstance(kernel_size, (list, tuple)) else kernel_size
        s = strides[0] if isinstance(strides, (list, tuple)) else strides
        d = dilation_rate[0] if isinstance(dilation_rate, (list, tuple)) else dilation_rate
        super().__init__(filters, k, init=kernel_initializer, activation=activation, border_mode=padding,
                         subsample_length=s, W_regularizer=kernel_regularizer, b_regularizer=bias_regularizer,
                         bias=use_bias, input_shape=input_shape, dilation=d, **kwargs)


class Conv2D(K1.Convolution2D):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", data_format=None, dilation_rate=(1, 1),
                 activation=None, use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zero",
                 kernel_regularizer=None, bias_regularizer=None, input_shape=None, **kwargs):
        ks = tuple(kernel_size) if isinstance(kernel_size, (list, tuple)) else (kernel_size, kernel_size)
        st = tuple(strides) if isinstance(strides, (list, tuple)) else (strides, strides)
        dl = tuple(dilation_rate) if isinstance(dilation_rate, (list, tuple)) else (dilation_rate, dilation_rate)
        K1.Layer.__init__(self, input_shape=input_shape, **kwargs)
        self._setup(filters, ks, kernel_initializer, activation, padding, st, _fmt(data_format), dl,
                    kernel_regularizer, bias_regularizer, use_bias)


class LocallyConnected1D(K1.LocallyConnected1D):
    def __init__(self, filters, kernel_size, strides=1, padding="valid", activation=None, use_bias=True,
                 kernel_regularizer=None, bias_regularizer=None, input_shape=None, **kwargs):
        k = kernel_size[0] if isinstance(kernel_size, (list, tuple)) else kernel_size
        s = strides[0] if isinstance(strides, (list, tuple)) else strides
        super().__init__(filters, k, activation=activation, border_mode=padding, subsample_length=s,
                         W_regularizer=kernel_regularizer, b_regularizer=bias_regularizer, bias=use_bias,
                         input_shape=input_shape, **kwargs)


class Cropping1D(K1.Cropping1D):
    pass


class MaxPooling1D(K1.MaxPooling1D):
    def __init__(self, pool_size=2, strides=None, padding="valid", input_shape=None, **kwargs):
        super().__init__(pool_size, strides, padding, input_shape=input_shape, **kwargs)


class AveragePooling1D(K1.AveragePooling1D):
    def __init__(self, pool_size=2, strides=None, padding="valid", input_shape=None, **kwargs):
        super().__init__(pool_size, strides, padding, input_shape=input_shape, **kwargs)


class GlobalAveragePooling1D(K1.GlobalAveragePooling1D):
    pass


class GlobalMaxPooling1D(K1.GlobalMaxPooling1D):
    pass


class GlobalAveragePooling2D(K1.GlobalAveragePooling2D):
    def __init__(self, data_format=None, input_shape=None, **kwargs):
        super().__init__(dim_ordering=_fmt(data_format), input_shape=input_shape, **kwargs)


class GlobalMaxPooling2D(K1.GlobalMaxPooling2D):
    def __init__(self, data_format=None, input_shape=None, **kwargs):
        super().__init__(dim_ordering=_fmt(data_format), input_shape=input_shape, **kwargs)


class GlobalAveragePooling3D(K1.GlobalAveragePooling3D):
    def __init__(self, data_format=None, input_shape=None, **kwargs):
        super().__init__(dim_ordering=_fmt(data_format), input_shape=input_shape, **kwargs)


class GlobalMaxPooling3D(K1.GlobalMaxPooling3D):
    def __init__(self, data_format=None, input_shape=None, **kwargs):
        super().__init__(dim_ordering=_fmt(data_format), input_shape=input_shape, **kwargs)


class Maximum(Merge):
    def __init__(self, input_shape=None, **kwargs):
        super().__init__(mode="max", input_shape=input_shape, **kwargs)


class Minimum(Merge):
    def __init__(self, input_shape=None, **kwargs):
        super().__init__(mode="min", input_shape=input_shape, **kwargs)


class Average(Merge):
    def __init__(self, input_shape=None, **kwargs):
        super().__init__(mode="ave", input_shape=input_shape, **kwargs)


def maximum(inputs, **kwargs):
    return Maximum(**kwargs)(inputs)


def minimum(inputs, **kwargs):
    return Minimum(**kwargs)(inputs)


def average(inputs, **kwargs):
    return Average(**kwargs)(inputs)
