"""Keras-2 API layers (keras2 layer specs / test_keras2_layers.py analogues):
shapes and numerics vs torch references, plus a small model that trains."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _seq(*layers):
    from zoo.pipeline.api.keras.models import Sequential
    m = Sequential()
    for l in layers:
        m.add(l)
    return m


def test_dense_and_conv2d_numerics():
    from zoo.pipeline.api.keras2.layers import Conv2D, Dense
    torch.manual_seed(0)
    d = Dense(5, activation="relu", input_shape=(7,))
    m = _seq(d)
    x = torch.randn(3, 7)
    assert torch.allclose(m(x), F.relu(F.linear(x, d.weight, d.bias)), atol=1e-5)
    c = Conv2D(4, (3, 3), strides=(2, 2), padding="same", data_format="channels_first", input_shape=(2, 9, 9))
    m2 = _seq(c)
    x = torch.randn(2, 2, 9, 9)
    y = m2(x)
    assert tuple(y.shape) == (2, 4, 5, 5)
    ref_w = torch.as_tensor(c.get_weights()[0])
    assert ref_w.numel() == 4 * 2 * 9


def test_pooling_merge_and_training():
    from zoo.pipeline.api.keras.engine.topology import Model
    from zoo.pipeline.api.keras.layers import Input
    from zoo.pipeline.api.keras2.layers import (Conv1D, Dense, Dropout, Flatten, GlobalMaxPooling1D, MaxPooling1D,
                                                Maximum, average)
    inp = Input(shape=(12, 4))
    a = Conv1D(6, 3, activation="relu")(inp)
    b = Conv1D(6, 3, activation="tanh")(inp)
    mx = Maximum()([a, b])
    av = average([a, b])
    h = MaxPooling1D(2)(mx)
    g = GlobalMaxPooling1D()(av)
    out = Dense(1)(Dropout(0.1)(Dense(8)(Flatten()(h))))
    m = Model(inp, [out, g])
    xs = np.random.rand(4, 12, 4).astype(np.float32)
    o1, o2 = m.predict(xs)
    assert o1.shape == (4, 1) and o2.shape == (4, 6)
    reg = Model(inp, out)
    y = xs.sum((1, 2)).reshape(-1, 1).astype(np.float32)
    reg.compile(optimizer="adam", loss="mse")
    before = reg.evaluate(xs, y)[0]
    reg.fit(xs, y, batch_size=4, nb_epoch=30)
    assert reg.evaluate(xs, y)[0] < before
