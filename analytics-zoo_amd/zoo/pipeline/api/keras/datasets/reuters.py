"""Reuters newswire topics (Py/pipeline/api/keras/datasets/reuters.py) from a local ``reuters.npz``."""
import numpy as np

from zoo.pipeline.api.keras.datasets._npz import load_npz, preprocess, sequences


def load_data(dest_dir="/tmp/.zoo/dataset", nb_words=None, oov_char=2, test_split=0.2, maxlen=None, skip_top=0):
    d = load_npz(dest_dir, "reuters.npz")
    if "x" in d or "x_flat" in d:
        x = preprocess(sequences(d, "x"), nb_words, skip_top, maxlen, oov_char=oov_char)
        y = d["y"]
        n = int(len(x) * (1 - test_split))
        return (x[:n], y[:n]), (x[n:], y[n:])
    return ((preprocess(sequences(d, "x_train"), nb_words, skip_top, maxlen, oov_char=oov_char), d["y_train"]),
            (preprocess(sequences(d, "x_test"), nb_words, skip_top, maxlen, oov_char=oov_char), d["y_test"]))


def pad(seqs, maxlen, value=0):
    out = np.full((len(seqs), maxlen), value, np.int64)
    for i, s in enumerate(seqs):
        s = s[-maxlen:]
        out[i, maxlen - len(s):] = s
    return out
