"""TextMatcher base (Zs/models/textmatching/TextMatcher.scala; Py text_matcher.py:24-60)."""
import numpy as np

from zoo.models.common.ranker import Ranker
from zoo.models.common.zoo_model import ZooModel


def prepare_embedding(embedding_file, word_index=None, randomize_unknown=False, normalize=False, seed=0):
    """GloVe text file -> [max_index + 1, dim] table (row 0 = padding/unknown)."""
    vecs, dim = {}, None
    with open(embedding_file, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip().split(" ")
            if len(parts) < 2:
                continue
            if word_index is None or parts[0] in word_index:
                vecs[parts[0]] = np.asarray(parts[1:], np.float32)
                dim = len(parts) - 1
    if word_index is None:
        word_index = {w: i + 1 for i, w in enumerate(sorted(vecs))}
    rng = np.random.default_rng(seed)
    table = np.zeros((max(word_index.values()) + 1, dim), np.float32)
    for w, i in word_index.items():
        if w in vecs:
            table[i] = vecs[w]
        elif randomize_unknown:
            table[i] = rng.uniform(-0.05, 0.05, dim)
    if normalize:
        n = np.linalg.norm(table, axis=1, keepdims=True)
        table = np.where(n > 0, table / np.maximum(n, 1e-12), table)
    return table


class TextMatcher(ZooModel, Ranker):
    def __init__(self, text1_length, vocab_size, embed_size=300, embed_weights=None, train_embed=True,
                 target_mode="ranking", **kwargs):
        super().__init__(**kwargs)
        if target_mode not in ("ranking", "classification"):
            raise ValueError("target_mode should be either ranking or classification")
        self.text1_length, self.vocab_size, self.embed_size = int(text1_length), int(vocab_size), int(embed_size)
        self.embed_weights, self.train_embed, self.target_mode = embed_weights, train_embed, target_mode
