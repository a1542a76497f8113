import os

import numpy as np


def load_npz(dest_dir, name):
    path = os.path.join(dest_dir, name)
    if not os.path.exists(path):
        raise FileNotFoundError("%s not found (no download: place the file there)" % path)
    with np.load(path, allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def sequences(d, key):
    """Padded 2-D array, or ``<key>_flat`` + ``<key>_lengths`` -> list of int arrays."""
    if key in d:
        return [np.asarray(r) for r in d[key]]
    flat, lens = d[key + "_flat"], d[key + "_lengths"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    return [flat[offs[i]:offs[i + 1]] for i in range(len(lens))]


def preprocess(seqs, nb_words=None, skip_top=0, maxlen=None, start_char=1, oov_char=2, index_from=3):
    out = []
    for s in seqs:
        s = [int(w) + index_from for w in s if int(w) != 0]
        if start_char is not None:
            s = [start_char] + s
        if nb_words is not None:
            s = [w if skip_top <= w < nb_words else oov_char for w in s]
        if maxlen is not None:
            s = s[:maxlen]
        out.append(np.asarray(s, np.int64))
    return out
