"""Boston housing regression (Py/pipeline/api/keras/datasets/boston_housing.py)."""
import numpy as np

from zoo.pipeline.api.keras.datasets._npz import load_npz


def load_data(dest_dir="/tmp/.zoo/dataset", test_split=0.2, seed=113):
    d = load_npz(dest_dir, "boston_housing.npz")
    x, y = d["x"], d["y"]
    rng = np.random.RandomState(seed)
    idx = np.arange(len(x))
    rng.shuffle(idx)
    x, y = x[idx], y[idx]
    n = int(len(x) * (1 - test_split))
    return (x[:n], y[:n]), (x[n:], y[n:])
