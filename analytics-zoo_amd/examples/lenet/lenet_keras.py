#!/usr/bin/env python3
"""LeNet-5 on MNIST through zoo.pipeline.api.keras (BASELINE config 1; reference:
Zs/examples/lenetLocal/Train.scala, pyzoo's keras LeNet quick start).

``--data DIR`` reads the MNIST idx files (train-images-idx3-ubyte, ...) from DIR; without it
the script trains on a synthetic MNIST-shaped set whose labels are a learnable function of
the image. Channels-first (``th``) Keras ordering, as in the reference example.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def build_lenet(classes=10):
    from zoo.pipeline.api.keras.layers import Convolution2D, Dense, Dropout, Flatten, MaxPooling2D, Reshape
    from zoo.pipeline.api.keras.models import Sequential
    m = Sequential()
    m.add(Reshape((1, 28, 28), input_shape=(28, 28, 1)))
    m.add(Convolution2D(6, 5, 5, activation="tanh", name="conv1_5x5"))
    m.add(MaxPooling2D())
    m.add(Convolution2D(12, 5, 5, activation="tanh", name="conv2_5x5"))
    m.add(MaxPooling2D())
    m.add(Flatten())
    m.add(Dense(100, activation="tanh", name="fc1"))
    m.add(Dropout(0.1))
    m.add(Dense(classes, activation="softmax", name="fc2"))
    return m


def synthetic_mnist(n, seed=0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 10, n)
    x = rng.random((n, 28, 28, 1)).astype(np.float32) * 0.2
    for i, c in enumerate(y):   # a bright bar whose position encodes the class
        x[i, 2 + 2 * c:4 + 2 * c, 4:24, 0] += 0.8
    return x, y


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data", default=None)
    ap.add_argument("--n", type=int, default=2048, help="synthetic set size")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--lr", type=float, default=0.01)
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("lenet5")
    if a.data:
        from zoo.pipeline.api.keras.datasets import mnist
        (x, y), (xt, yt) = mnist.load_data(a.data)
        x = (x.reshape(-1, 28, 28, 1) / 255.0).astype(np.float32)
        xt = (xt.reshape(-1, 28, 28, 1) / 255.0).astype(np.float32)
    else:
        x, y = synthetic_mnist(a.n)
        xt, yt = synthetic_mnist(max(256, a.n // 8), seed=1)
    m = build_lenet()
    m.compile(optimizer=Adam(lr=a.lr), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    m.fit(x, y, batch_size=a.batch, nb_epoch=a.epochs, validation_data=(xt, yt))
    res = m.evaluate(xt, yt, batch_size=a.batch)
    print("test loss/accuracy:", res)
    return res


if __name__ == "__main__":
    main()
