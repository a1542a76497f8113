#!/usr/bin/env python3
"""NNFrames image transfer learning (pyzoo/zoo/examples/nnframes/imageTransferLearning,
Zs/examples/nnframes/imageTransferLearning): images read into a DataFrame with
NNImageReader, a frozen feature extractor (here a small random conv net standing in for a
pretrained backbone -- no model download) + a trainable classifier head fitted with
NNClassifier, predictions added as a DataFrame column. ``--images DIR`` with one
sub-directory per class, or synthetic PNGs written to a temp dir."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def write_synthetic(root, per_class=24, size=32):
    from PIL import Image
    rng = np.random.default_rng(0)
    for c, color in enumerate(((220, 40, 40), (40, 40, 220))):
        d = os.path.join(root, "class%d" % c)
        os.makedirs(d, exist_ok=True)
        for i in range(per_class):
            img = (rng.random((size, size, 3)) * 60 + np.array(color) * 0.7).astype(np.uint8)
            Image.fromarray(img).save(os.path.join(d, "%d.png" % i))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--images", default=None)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--epochs", type=int, default=10)
    a = ap.parse_args(argv)
    import torch
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.nnframes import NNClassifier, NNImageReader
    init_nncontext("image_transfer_learning")
    tmp = None
    root = a.images
    if root is None:
        tmp = tempfile.TemporaryDirectory()
        root = tmp.name
        write_synthetic(root, size=a.size)
    frames = []
    for c, sub in enumerate(sorted(os.listdir(root))):
        df = NNImageReader.readImages(os.path.join(root, sub), resizeH=a.size, resizeW=a.size)
        df["label"] = float(c + 1)
        frames.append(df)
    import pandas as pd
    df = pd.concat(frames, ignore_index=True)
    # frozen "backbone": mean colour per channel + a fixed random projection of the pixels
    torch.manual_seed(0)
    proj = torch.randn(a.size * a.size * 3, 13)

    def features(row):
        img = np.frombuffer(row["image"]["data"], np.uint8).reshape(a.size, a.size, -1)[..., :3]
        x = torch.from_numpy(img.astype(np.float32) / 255.0)
        return np.concatenate([x.mean((0, 1)).numpy(), (x.reshape(-1) @ proj).numpy() / 50.0]).astype(np.float32)
    df["features"] = df.apply(features, axis=1)
    head = Sequential()
    head.add(Dense(2, activation="log_softmax", input_shape=(16,)))
    clf = NNClassifier(head, ClassNLLCriterion(), [16]).setBatchSize(16).setMaxEpoch(a.epochs) \
        .setOptimMethod(Adam(lr=0.05))
    model = clf.fit(df)
    out = model.transform(df)
    acc = float((out["prediction"].values == df["label"].values).mean())
    print("train accuracy:", acc)
    if tmp is not None:
        tmp.cleanup()
    return acc


if __name__ == "__main__":
    main()
