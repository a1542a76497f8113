#!/usr/bin/env python3
"""Train a PyTorch module through the Zoo Keras API (pyzoo/zoo/examples/pytorch/train/
SimpleTrainingExample.py): TorchNet.from_pytorch wraps the module, TorchCriterion the
loss, then compile / fit / evaluate / predict run on the framework's engine (native kernels
where the module's ops have them, on the GPU when present)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--epochs", type=int, default=20)
    a = ap.parse_args(argv)
    import torch
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.net import TorchCriterion, TorchNet
    init_nncontext("pytorch_simple")
    torch.manual_seed(0)
    mod = torch.nn.Sequential(torch.nn.Linear(2, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1))
    net = TorchNet.from_pytorch(mod, input_shape=(2,))
    rng = np.random.default_rng(0)
    x = rng.random((a.n, 2)).astype(np.float32)
    y = ((x[:, :1] * x[:, 1:]) > 0.25).astype(np.float32)
    net.compile(optimizer="adam", loss=TorchCriterion.from_pytorch(torch.nn.BCEWithLogitsLoss()))
    before = net.evaluate(x, y)[0]
    net.fit(x, y, batch_size=32, nb_epoch=a.epochs)
    after = net.evaluate(x, y)[0]
    print("loss %.4f -> %.4f" % (before, after))
    return before, after


if __name__ == "__main__":
    main()
