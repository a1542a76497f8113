"""Feature helpers for the recommendation models (Py/models/recommendation/utils.py,
Zs/models/recommendation/Utils.scala). Rows are dicts / pandas rows."""
import hashlib

import numpy as np

from zoo.models.recommendation.recommender import UserItemFeature


def hash_bucket(content, bucket_size=1000, start=0):
    """Stable bucket id of a string (md5, unlike Python's salted hash)."""
    h = int(hashlib.md5(str(content).encode()).hexdigest(), 16)
    return h % bucket_size + start


def categorical_from_vocab_list(sth, vocab_list, default=-1, start=0):
    return vocab_list.index(sth) + start if sth in vocab_list else default


def get_boundaries(target, boundaries, default=-1, start=0):
    if target == "?":
        return default
    for i, b in enumerate(boundaries):
        if target < b:
            return i + start
    return len(boundaries) + start


def get_negative_samples(indexed, neg_num=1, item_count=None, seed=0):
    """(user, item, label=2) positives + ``neg_num`` random (user, item', label=1) negatives per positive."""
    rng = np.random.default_rng(seed)
    pos = {(int(u), int(i)) for u, i, *_ in indexed}
    items = item_count or max(i for _, i in pos)
    out = []
    for u, i in sorted(pos):
        out.append((u, i, 2))
        for _ in range(neg_num):
            while True:
                j = int(rng.integers(1, items + 1))
                if (u, j) not in pos:
                    break
            out.append((u, j, 1))
    return out


def _global(row, cols, dims):
    acc, out = 0, []
    for c, d in zip(cols, dims):
        out.append(acc + int(row[c]))
        acc += d
    return out


def get_wide_tensor(row, column_info):
    """Global indices of the wide (base + cross) columns: the WideAndDeep wide input."""
    ci = column_info
    return np.array(_global(row, ci.wide_base_cols + ci.wide_cross_cols, ci.wide_base_dims + ci.wide_cross_dims),
                    np.float32)


def get_deep_tensors(row, column_info):
    ci = column_info
    out = []
    if ci.indicator_cols:
        ind = np.zeros(sum(ci.indicator_dims), np.float32)
        ind[_global(row, ci.indicator_cols, ci.indicator_dims)] = 1.0
        out.append(ind)
    if ci.embed_cols:
        out.append(np.array([float(row[c]) for c in ci.embed_cols], np.float32))
    if ci.continuous_cols:
        out.append(np.array([float(row[c]) for c in ci.continuous_cols], np.float32))
    if not out:
        raise TypeError("Empty deep tensors")
    return out


def row_to_sample(row, column_info, model_type="wide_n_deep"):
    wide = get_wide_tensor(row, column_info)
    deep = get_deep_tensors(row, column_info)
    label = float(row[column_info.label])
    mt = model_type.lower()
    if mt == "wide_n_deep":
        feats = [wide] + deep
    elif mt == "wide":
        feats = [wide]
    elif mt == "deep":
        feats = deep
    else:
        raise TypeError("Unsupported model_type: %s" % model_type)
    return feats, label


def to_user_item_feature(row, column_info, model_type="wide_n_deep"):
    return UserItemFeature(row["userId"], row["itemId"], row_to_sample(row, column_info, model_type))


def samples_to_arrays(samples):
    """[(feats list, label)] -> ([stacked arrays per input], labels array)."""
    n_in = len(samples[0][0])
    xs = [np.stack([s[0][i] for s in samples]) for i in range(n_in)]
    return xs, np.array([s[1] for s in samples], np.float32)
