#!/usr/bin/env python3
"""TFPark KerasModel on ndarrays and on a TFDataset (pyzoo/zoo/examples/tensorflow/tfpark/
keras/keras_ndarray.py and keras_dataset.py): a Keras-style MNIST MLP trained with
KerasModel.fit on ndarrays (or, with ``--use-dataset``, on a TFDataset), then evaluated."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--use-dataset", action="store_true", help="feed a TFDataset instead of ndarrays")
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.layers import Dense, Dropout, Flatten
    from zoo.pipeline.api.keras.models import Sequential
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.tfpark import KerasModel, TFDataset
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lenet"))
    from lenet_keras import synthetic_mnist
    init_nncontext("tfpark_keras")
    x, y = synthetic_mnist(a.n)
    m = Sequential()
    m.add(Flatten(input_shape=(28, 28, 1)))
    m.add(Dense(64, activation="relu"))
    m.add(Dropout(0.2))
    m.add(Dense(10, activation="softmax"))
    km = KerasModel(m, optimizer=Adam(lr=0.003), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    if a.use_dataset:
        km.fit(TFDataset.from_ndarrays((x, y), batch_size=a.batch), epochs=a.epochs)
    else:
        km.fit(x, y, batch_size=a.batch, epochs=a.epochs)
    res = km.evaluate(x, y, batch_per_thread=a.batch)
    print("evaluate:", res)
    return res


if __name__ == "__main__":
    main()
