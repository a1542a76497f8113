"""ImageClassifier / ImageModel / ImageConfigure (Zs/models/image/imageclassification/
ImageClassifier.scala:37-53, ImageClassificationConfig.scala:56-190, Zs/models/image/common/
ImageModel.scala:35-164, ImageConfigure; Py imageclassification/image_classifier.py).

``ImageClassifier(model_name)`` builds the named backbone; ``predict_image_set``
applies the model's configured preprocessing (resize -> center crop ->
channel normalize -> CHW, per ImageClassificationConfig) and stores
``predict`` = [(class, probability)] sorted descending (LabelOutput).
"""
import numpy as np
import torch

from zoo.models.common.zoo_model import ZooModel
from zoo.models.image.imageclassification import nets

IMAGENET_MEAN_RGB = (123.0, 117.0, 104.0)

# name -> (resize short side, crop, mean R,G,B, scale); ImageClassificationConfig.scala
_CONFIGS = {
    "alexnet": (256, 227, IMAGENET_MEAN_RGB, 1.0), "inception-v1": (256, 224, IMAGENET_MEAN_RGB, 1.0),
    "inception-v3": (342, 299, (127.5, 127.5, 127.5), 1 / 127.5), "resnet-50": (256, 224, IMAGENET_MEAN_RGB, 1.0),
    "vgg-16": (256, 224, IMAGENET_MEAN_RGB, 1.0), "vgg-19": (256, 224, IMAGENET_MEAN_RGB, 1.0),
    "densenet-161": (256, 224, (123.68, 116.78, 103.94), 0.017), "squeezenet": (256, 227, IMAGENET_MEAN_RGB, 1.0),
    "mobilenet": (256, 224, (123.68, 116.78, 103.94), 0.017), "mobilenet-v2": (256, 224, (123.68, 116.78, 103.94),
                                                                              0.017)}


class ImageConfigure:
    def __init__(self, pre_processor=None, post_processor=None, batch_per_partition=4, label_map=None):
        self.pre_processor, self.post_processor = pre_processor, post_processor
        self.batch_per_partition, self.label_map = batch_per_partition, label_map

    @staticmethod
    def for_model(name, label_map=None):
        from zoo.feature.common import ChainedPreprocessing
        from zoo.feature.image import (ImageAspectScale, ImageCenterCrop, ImageChannelScaledNormalizer,
                                       ImageMatToTensor)
        key = next((k for k in _CONFIGS if name.lower().startswith(k)), "resnet-50")
        size, crop, mean, scale = _CONFIGS[key]
        pre = ChainedPreprocessing([ImageAspectScale(size, max_size=10 ** 6), ImageCenterCrop(crop, crop),
                                    ImageChannelScaledNormalizer(mean[0], mean[1], mean[2], scale),
                                    ImageMatToTensor(to_RGB=True)])
        return ImageConfigure(pre, LabelOutput(label_map), 4, label_map)


class LabelOutput:
    """Top-k (class, probability) per image (LabelOutput.scala)."""

    def __init__(self, label_map=None, clses="clses", probs="probs", prob_as_output=True, top_k=5):
        self.label_map, self.top_k = label_map, top_k

    def __call__(self, scores):
        p = np.asarray(scores, np.float64)
        if p.min() < 0 or abs(p.sum() - 1.0) > 1e-3:
            e = np.exp(p - p.max())
            p = e / e.sum()
        idx = np.argsort(-p, kind="stable")[:self.top_k]
        lab = (lambda i: self.label_map.get(int(i), str(int(i)))) if self.label_map else (lambda i: int(i))
        return [(lab(i), float(p[i])) for i in idx]


class ImageModel(ZooModel):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.config = None

    def get_config(self):
        return self.config

    @torch.no_grad()
    def predict_image_set(self, image_set, configure=None, batch_size=32):
        cfg = configure or self.config
        if getattr(self, "int8", False):
            from zoo.ops.quant import is_quantized
            if not is_quantized(self):
                self.quantize()  # "*-int8" / "*-quantize" configs serve the int8 model
        s = image_set.transform(cfg.pre_processor) if cfg is not None and cfg.pre_processor else image_set
        x = np.stack([f["imageTensor"] for f in s.features]).astype(np.float32)
        out = self.predict(x, batch_size=batch_size)
        post = cfg.post_processor if cfg is not None else None
        for f, o in zip(s.features, out):
            f["predict"] = post(o) if post is not None else o
        return s


class ImageClassifier(ImageModel):
    def __init__(self, model_name="resnet-50", num_classes=1000, label_map=None, **kwargs):
        super().__init__(**kwargs)
        self.model_name = model_name
        self.num_classes = int(num_classes)
        self.config = ImageConfigure.for_model(model_name, label_map)
        self.net = nets.build(model_name, num_classes)
        self.int8 = model_name.lower().endswith(("-int8", "-quantize"))
        self.built = True

    def build_model(self):
        return self.net

    def forward(self, x, *rest):
        return self.net(x)

    def call(self, x):
        return self.net(x)

    def _layer_list(self):
        return []

    @staticmethod
    def load_model(path, weight_path=None):
        from zoo.utils.checkpoint import load_object
        d = load_object(path)
        m = ImageClassifier(d["model_name"], d["num_classes"], d.get("label_map"))
        m.net.load_state_dict(d["state"])
        return m

    def save_model(self, path, weight_path=None, over_write=False):
        from zoo.utils.checkpoint import save_object
        save_object({"model_name": self.model_name, "num_classes": self.num_classes,
                     "label_map": self.config.label_map,
                     "state": {k: v.detach().cpu() for k, v in self.net.state_dict().items()}}, path, over_write)
