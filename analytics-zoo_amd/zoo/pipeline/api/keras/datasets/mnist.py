"""MNIST from local IDX files (Py/pipeline/api/keras/datasets/mnist.py)."""
import gzip
import os

import numpy as np

FILES = {"train_x": "train-images-idx3-ubyte", "train_y": "train-labels-idx1-ubyte",
         "test_x": "t10k-images-idx3-ubyte", "test_y": "t10k-labels-idx1-ubyte"}
TRAIN_MEAN, TRAIN_STD = 0.13066047740239506 * 255, 0.3081078 * 255


def read_idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    ndim = magic & 0xFF
    dtype = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}[(magic >> 8) & 0xFF]
    shape = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=dtype, offset=4 + 4 * ndim).reshape(shape)


def write_idx(path, arr):
    arr = np.ascontiguousarray(arr, np.uint8)
    head = bytes([0, 0, 0x08, arr.ndim]) + b"".join(int(d).to_bytes(4, "big") for d in arr.shape)
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "wb") as f:
        f.write(head + arr.tobytes())


def _find(dest_dir, name):
    for cand in (name, name + ".gz", name.replace("-idx", ".idx")):
        p = os.path.join(dest_dir, cand)
        if os.path.exists(p):
            return p
    raise FileNotFoundError("%s not found in %s (no download: place the MNIST files there)" % (name, dest_dir))


def read_data_sets(train_dir, data_type="train"):
    x = read_idx(_find(train_dir, FILES[data_type + "_x"]))
    y = read_idx(_find(train_dir, FILES[data_type + "_y"]))
    return x, y


def load_data(location="/tmp/.zoo/dataset/mnist"):
    """((x_train, y_train), (x_test, y_test)), images [N, 28, 28] uint8."""
    return read_data_sets(location, "train"), read_data_sets(location, "test")
