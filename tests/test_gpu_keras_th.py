"""The default Keras image ordering ("th", NCHW) runs on the native NHWC kernels:
channels-last memory propagates between layers (free permutes), and a LeNet and a
small BN ResNet-style model train with no MIOpen kernel in the GPU trace
(torch.profiler kernel names)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

BANNED = ("miopen", "MIOpen", "mlo", "naive_conv", "gridwise_", "Cijk_")


def _lenet():
    from zoo.pipeline.api.keras import layers as L
    from zoo.pipeline.api.keras.models import Sequential
    m = Sequential()
    m.add(L.Convolution2D(6, 5, 5, activation="tanh", input_shape=(1, 28, 28)))
    m.add(L.MaxPooling2D())
    m.add(L.Convolution2D(12, 5, 5, activation="tanh"))
    m.add(L.MaxPooling2D())
    m.add(L.Flatten())
    m.add(L.Dense(100, activation="tanh"))
    m.add(L.Dense(10, activation="softmax"))
    return m


def _small_resnet():
    from zoo.pipeline.api.keras import layers as L
    from zoo.pipeline.api.keras.base import Input
    from zoo.pipeline.api.keras.engine.topology import Model
    x = Input(shape=(3, 32, 32))
    h = L.Convolution2D(16, 3, 3, border_mode="same")(x)
    h = L.BatchNormalization()(h)
    h = L.Activation("relu")(h)
    r = L.Convolution2D(16, 3, 3, border_mode="same")(h)
    r = L.BatchNormalization()(r)
    h = L.Activation("relu")(L.merge([h, r], mode="sum"))
    h = L.AveragePooling2D()(h)
    h = L.Convolution2D(32, 3, 3, border_mode="same", activation="relu")(h)
    h = L.GlobalAveragePooling2D()(h)
    return Model(x, L.Dense(10, activation="softmax")(h))


def _kernels_of(fn):
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return [e.name for e in prof.events() if e.device_type.name == "CUDA"]


@pytest.mark.parametrize("make,shape", [(_lenet, (1, 28, 28)), (_small_resnet, (3, 32, 32))])
def test_keras_th_model_trains_without_miopen(gpu, make, shape):
    from zoo.common.nncontext import init_nncontext
    init_nncontext()
    torch.manual_seed(0)
    m = make()
    m.compile("adam", "sparse_categorical_crossentropy", ["accuracy"])
    rs = np.random.RandomState(0)
    y = rs.randint(0, 10, 512)
    x = rs.randn(512, *shape).astype(np.float32) * 0.5
    x[:, 0] += (y[:, None, None] - 4.5) * 0.3   # learnable signal (survives global pooling)
    m.fit(x, y, batch_size=64, nb_epoch=1)
    names = _kernels_of(lambda: m.fit(x, y, batch_size=64, nb_epoch=1))
    assert any("zoo::" in n for n in names)
    bad = sorted({n for n in names if any(b in n for b in BANNED)})
    assert not bad, bad[:5]
    m.fit(x, y, batch_size=64, nb_epoch=6)
    acc = m.evaluate(x, y, batch_size=128)[0]
    assert acc > 0.3, acc


def test_th_conv_output_is_channels_last_view(gpu):
    from zoo.pipeline.api.keras import layers as L
    from zoo.pipeline.api.keras.models import Sequential
    m = Sequential()
    m.add(L.Convolution2D(16, 3, 3, input_shape=(8, 12, 12)))
    m.add(L.Convolution2D(16, 3, 3))
    m = m.cuda()
    y = m(torch.randn(2, 8, 12, 12, device=gpu))
    assert y.shape == (2, 16, 8, 8)
    assert y.is_contiguous(memory_format=torch.channels_last)
