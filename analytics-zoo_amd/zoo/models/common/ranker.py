"""Ranker: NDCG / MAP evaluation for text matching models (Zs/models/common/Ranker.scala:37-175)."""
import numpy as np


def _ndcg(scores, labels, k):
    order = np.argsort(-scores)
    gains = (2.0 ** labels[order] - 1.0)[:k]
    disc = 1.0 / np.log2(np.arange(2, len(gains) + 2))
    dcg = float((gains * disc).sum())
    ideal = (2.0 ** np.sort(labels)[::-1] - 1.0)[:k]
    idcg = float((ideal * disc[: len(ideal)]).sum())
    return dcg / idcg if idcg > 0 else 0.0


def _map(scores, labels):
    order = np.argsort(-scores)
    rel = labels[order] > 0
    if rel.sum() == 0:
        return 0.0
    hits = np.cumsum(rel)
    return float((hits[rel] / (np.nonzero(rel)[0] + 1)).mean())


class Ranker:
    """Mixin/utility: evaluate ranking quality of a model over grouped
    (query, candidates) samples given as a list of (x, labels) pairs."""

    def evaluate_ndcg(self, groups, k):
        vals = []
        for x, labels in groups:
            s = np.asarray(self.predict(x)).reshape(-1)
            vals.append(_ndcg(s, np.asarray(labels, dtype=np.float64).reshape(-1), k))
        return float(np.mean(vals)) if vals else 0.0

    def evaluate_map(self, groups):
        vals = []
        for x, labels in groups:
            s = np.asarray(self.predict(x)).reshape(-1)
            vals.append(_map(s, np.asarray(labels).reshape(-1)))
        return float(np.mean(vals)) if vals else 0.0
