#!/usr/bin/env python3
"""Image classification inference (pyzoo/zoo/examples/imageclassification/predict.py): read a
folder of images into an ImageSet, run a zoo ImageClassifier (its model config supplies the
resize / crop / normalise pre-processing and the top-N LabelOutput post-processing) and print
the top classes of every image. Without --folder a few synthetic JPEGs are written first;
without a --model-path the backbone is randomly initialised (native NHWC bf16 kernels on the
GPU, the fp32 reference path on the CPU)."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def _write_images(d, n, seed):
    from PIL import Image
    rng = np.random.default_rng(seed)
    for i in range(n):
        Image.fromarray(rng.integers(0, 255, (96, 128, 3), dtype=np.uint8)).save(os.path.join(d, "img%d.jpg" % i))


def main(argv=None):
    ap = _common.add_common(argparse.ArgumentParser(description=__doc__.split("\n")[0]))
    ap.add_argument("--folder", default=None)
    ap.add_argument("--model", default="squeezenet", help="ImageClassifier model name (e.g. resnet-50, mobilenet)")
    ap.add_argument("--model-path", default=None)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--images", type=int, default=3)
    ap.add_argument("--topn", type=int, default=3)
    a = ap.parse_args(argv)
    import torch
    from zoo.feature.image.imageset import ImageSet
    from zoo.models.image.imageclassification.image_classifier import ImageClassifier
    torch.manual_seed(a.seed)
    with tempfile.TemporaryDirectory() as tmp:
        folder = a.folder
        if folder is None:
            folder = tmp
            _write_images(folder, a.images, a.seed)
        model = ImageClassifier.load_model(a.model_path) if a.model_path else \
            ImageClassifier(a.model, a.classes, label_map={i: "class_%d" % i for i in range(a.classes)})
        model.eval()
        if torch.cuda.is_available():
            model = model.cuda()
        model.config.post_processor.top_k = a.topn
        out = model.predict_image_set(ImageSet.read(folder))
        res = {}
        for f in out.features:
            res[os.path.basename(str(f.get("uri", f.get("path", "?"))))] = f["predict"]
        for k in sorted(res):
            print(k, res[k])
        return res


if __name__ == "__main__":
    main()
