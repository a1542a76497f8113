"""ImageSet (Py/feature/image/imageset.py:21-215, Zs/feature/image/ImageSet.scala).

``LocalImageSet`` holds ImageFeature dicts in memory; ``DistributedImageSet``
is the per-rank shard (rank::world of the file list) used by one process per
GPU. ``read(path, with_label=True)`` labels images by their class folder
(sorted folder names, one-based by default, like the reference).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from zoo.pipeline.nnframes.nn_image_reader import _list, decode_image


class ImageSet:
    def __init__(self, features, label_map=None):
        self.features = list(features)
        self._label_map = label_map

    # ---- construction -------------------------------------------------------------
    @classmethod
    def read(cls, path, sc=None, min_partitions=1, resize_height=-1, resize_width=-1, image_codec=-1,
             with_label=False, one_based_label=True, distributed=False, num_threads=8):
        label_map = None
        if with_label:
            classes = sorted(d for d in os.listdir(path) if os.path.isdir(os.path.join(path, d)))
            label_map = {c: i + (1 if one_based_label else 0) for i, c in enumerate(classes)}
            files = [(f, label_map[c]) for c in classes for f in _list(os.path.join(path, c))]
        else:
            files = [(f, None) for f in _list(path)]
        if distributed:
            from zoo.common.nncontext import get_nncontext
            ctx = get_nncontext()
            files = files[ctx.rank::ctx.world_size]

        def load(item):
            f, lab = item
            with open(f, "rb") as fh:
                raw = fh.read()
            arr = decode_image(raw, resize_height, resize_width, image_codec)
            feat = {"uri": f, "bytes": raw, "mat": arr.astype(np.float32), "originalSize": arr.shape}
            if lab is not None:
                feat["label"] = np.array([lab], np.float32)
            return feat
        with ThreadPoolExecutor(num_threads) as ex:
            feats = list(ex.map(load, files))
        klass = DistributedImageSet if distributed else LocalImageSet
        return klass(feats, label_map)

    @classmethod
    def read_sequence_files(cls, path, sc=None, min_partitions=1, class_num=1000, distributed=False):
        """Images with labels from Hadoop SequenceFiles in ``path`` (a file or a folder),
        as written by BigDL's ImageNet sequence-file generator (ImageSet.scala:335-352):
        records with label > ``class_num`` are dropped; pixels stay BGR like the reference."""
        from zoo.feature.image.sequence_file import decode_image_record, read_sequence_file
        files = [path] if os.path.isfile(path) else sorted(
            os.path.join(path, f) for f in os.listdir(path) if not f.startswith((".", "_")))
        if distributed:
            from zoo.common.nncontext import get_nncontext
            ctx = get_nncontext()
            files = files[ctx.rank::ctx.world_size]
        feats = []
        for fp in files:
            for k, v in read_sequence_file(fp):
                label, name, img = decode_image_record(k, v)
                if label > class_num:
                    continue
                feats.append({"uri": name, "mat": img.astype(np.float32), "originalSize": img.shape,
                              "label": np.array([label], np.float32)})
        return (DistributedImageSet if distributed else LocalImageSet)(feats)

    readSequenceFiles = read_sequence_files

    @classmethod
    def from_arrays(cls, images, labels=None):
        feats = []
        for i, im in enumerate(images):
            im = np.asarray(im)
            im = im[:, :, None] if im.ndim == 2 else im
            f = {"uri": str(i), "mat": im.astype(np.float32), "originalSize": im.shape}
            if labels is not None:
                f["label"] = np.array([labels[i]], np.float32).reshape(-1)
            feats.append(f)
        return LocalImageSet(feats)

    # ---- API ------------------------------------------------------------------------
    def is_local(self):
        return not isinstance(self, DistributedImageSet)

    def is_distributed(self):
        return isinstance(self, DistributedImageSet)

    @property
    def label_map(self):
        return self._label_map

    def get_label_map(self):
        return self._label_map

    def transform(self, transformer):
        return type(self)([transformer.apply(dict(f)) for f in self.features], self._label_map)

    def __rshift__(self, transformer):
        return self.transform(transformer)

    def get_image(self, key="floats", to_chw=True):
        out = []
        for f in self.features:
            if key in f and key != "floats":
                out.append(f[key])
                continue
            m = f.get("imageTensor") if key == "imageTensor" else f["mat"]
            out.append(m.transpose(2, 0, 1) if to_chw and m.ndim == 3 and key != "imageTensor" else m)
        return out

    def get_label(self):
        return [f.get("label") for f in self.features]

    def get_predict(self, key="predict"):
        return [(f.get("uri"), f.get(key)) for f in self.features]

    def __len__(self):
        return len(self.features)

    def to_featureset(self, batch_size=32, shuffle=True):
        """Stack ``imageTensor`` (or CHW ``mat``) + ``label`` into a FeatureSet."""
        from zoo.feature.common import FeatureSet
        x = np.stack([f["imageTensor"] if "imageTensor" in f else f["mat"].transpose(2, 0, 1)
                      for f in self.features]).astype(np.float32)
        labels = [f.get("label") for f in self.features]
        y = None if any(l is None for l in labels) else np.concatenate(labels).astype(np.float32)
        return FeatureSet.from_ndarrays(x, y, batch_size, shuffle=shuffle)

    def to_batch_u8(self):
        """Same-size images as one uint8 [N, H, W, C] array (input of the GPU resize kernel)."""
        return np.stack([np.clip(f["mat"], 0, 255).astype(np.uint8) for f in self.features])


class LocalImageSet(ImageSet):
    pass


class DistributedImageSet(ImageSet):
    pass
