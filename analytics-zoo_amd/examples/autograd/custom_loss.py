#!/usr/bin/env python3
"""Custom loss and custom layer with zoo.pipeline.api.autograd (pyzoo/zoo/examples/
autograd/customloss.py and custom.py): a mean-absolute-error loss written with autograd
ops and a Lambda layer, trained on a synthetic linear problem."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def mean_absolute_error(y_true, y_pred):
    import zoo.pipeline.api.autograd as A
    return A.mean(A.abs(y_true - y_pred), axis=1)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--epochs", type=int, default=10)
    a = ap.parse_args(argv)
    import zoo.pipeline.api.autograd as A
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.autograd import CustomLoss, Lambda
    from zoo.pipeline.api.keras.layers import Dense, Input
    from zoo.pipeline.api.keras.models import Model
    from zoo.pipeline.api.keras.optimizers import SGD
    init_nncontext("autograd")
    rng = np.random.default_rng(0)
    x = rng.random((a.n, 2)).astype(np.float32)
    y = (2 * x[:, :1] + 3 * x[:, 1:] + 0.4).astype(np.float32)
    inp = Input(shape=(2,))
    scaled = Lambda(lambda t: t * 2.0 + A.epsilon())(inp)         # a custom (autograd) layer
    out = Dense(1)(scaled)
    m = Model(inp, out)
    m.compile(optimizer=SGD(learningrate=0.1), loss=CustomLoss(mean_absolute_error, y_pred_shape=[1],
                                                               y_true_shape=[1]))
    m.fit(x, y, batch_size=32, nb_epoch=a.epochs)
    err = float(np.abs(m.predict(x).reshape(-1) - y.reshape(-1)).mean())
    print("mean absolute error:", err)
    return err


if __name__ == "__main__":
    main()
