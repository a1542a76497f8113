"""NNImageReader / NNImageSchema (Zs/pipeline/nnframes/NNImageReader.scala:35-182,
Py/pipeline/nnframes/nn_image_reader.py:25-54, nn_image_schema.py:25).

Reads a directory / glob of images into a pandas DataFrame whose ``image``
column holds the Spark-ML image struct: origin, height, width, nChannels,
mode (OpenCV type code: 16 = CV_8UC3, 0 = CV_8UC1, 24 = CV_8UC4) and data
(row-major HWC bytes, BGR channel order like the reference's OpenCV decode).
Decoding uses PIL with a thread pool.
"""
import glob
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".gif", ".ppm", ".tif", ".tiff", ".webp")
_MODE = {1: 0, 3: 16, 4: 24}


def _list(path):
    if os.path.isdir(path):
        out = []
        for root, _, files in os.walk(path):
            out.extend(os.path.join(root, f) for f in files if f.lower().endswith(_EXT))
        return sorted(out)
    return sorted(glob.glob(path))


def decode_image(path_or_bytes, resize_h=-1, resize_w=-1, image_codec=-1):
    """bytes/path -> HWC uint8 BGR array (gray kept 1-channel when image_codec == 0)."""
    import io
    from PIL import Image
    src = io.BytesIO(path_or_bytes) if isinstance(path_or_bytes, (bytes, bytearray)) else path_or_bytes
    with Image.open(src) as im:
        if image_codec == 0 or im.mode in ("L", "1", "I;16") and image_codec != 1:
            im = im.convert("L")
        elif im.mode == "RGBA" and image_codec == -1:
            pass
        else:
            im = im.convert("RGB")
        if resize_h > 0 and resize_w > 0:
            im = im.resize((resize_w, resize_h), Image.BILINEAR)
        arr = np.asarray(im, dtype=np.uint8)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    elif arr.shape[2] == 3:
        arr = arr[:, :, ::-1]
    elif arr.shape[2] == 4:
        arr = arr[:, :, [2, 1, 0, 3]]
    return np.ascontiguousarray(arr)


def image_row(origin, arr):
    h, w, c = arr.shape
    return {"origin": origin, "height": int(h), "width": int(w), "nChannels": int(c), "mode": _MODE.get(c, 16),
            "data": arr.tobytes()}


def row_to_array(row):
    return np.frombuffer(row["data"], dtype=np.uint8).reshape(row["height"], row["width"], row["nChannels"])


class NNImageReader:
    @staticmethod
    def readImages(path, sc=None, minPartitions=1, resizeH=-1, resizeW=-1, image_codec=-1,  # noqa: N802,N803
                   num_threads=8):
        import pandas as pd
        files = _list(path)
        with ThreadPoolExecutor(num_threads) as ex:
            arrs = list(ex.map(lambda f: decode_image(f, resizeH, resizeW, image_codec), files))
        return pd.DataFrame({"image": [image_row(f, a) for f, a in zip(files, arrs)]})


def with_origin_column(dataset, imageColumn="image", originColumn="origin"):  # noqa: N803
    out = dataset.copy()
    out[originColumn] = [r["origin"] for r in dataset[imageColumn]]
    return out
