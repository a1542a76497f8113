"""IMDB reviews (Py/pipeline/api/keras/datasets/imdb.py) from a local ``imdb.npz``."""
from zoo.pipeline.api.keras.datasets._npz import load_npz, preprocess, sequences


def load_data(dest_dir="/tmp/.zoo/dataset", nb_words=None, oov_char=2, maxlen=None, skip_top=0):
    d = load_npz(dest_dir, "imdb.npz")
    xtr = preprocess(sequences(d, "x_train"), nb_words, skip_top, maxlen, oov_char=oov_char)
    xte = preprocess(sequences(d, "x_test"), nb_words, skip_top, maxlen, oov_char=oov_char)
    return (xtr, d["y_train"]), (xte, d["y_test"])


def get_word_index(dest_dir="/tmp/.zoo/dataset", filename="imdb_word_index.json"):
    import json
    import os
    with open(os.path.join(dest_dir, filename)) as f:
        return json.load(f)
