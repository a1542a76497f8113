"""TextSet / TextFeature and text transformers (Zs/feature/text/*.scala:
TextSet.scala (word index generation 657-690, relation pairs/lists 399-520),
Tokenizer, Normalizer, WordIndexer, SequenceShaper, TextFeatureToSample;
Py/feature/text/text_set.py:23-470, transformer.py:28-150).

A TextFeature is a dict: ``uri``, ``text``, ``label``, ``tokens``,
``indices``, ``sample``, ``predict``. DistributedTextSet is the per-rank
shard (rank::world) for one-process-per-GPU jobs.
"""
import csv
import os
import re

import numpy as np

from zoo.feature.common import Preprocessing


def TextFeature(text=None, label=None, uri=None):  # noqa: N802 - reference name
    f = {"text": text, "uri": uri}
    if label is not None:
        f["label"] = int(label)
    return f


class Relation:
    def __init__(self, id1, id2, label):
        self.id1, self.id2, self.label = str(id1), str(id2), int(label)

    def __repr__(self):
        return "Relation(%s, %s, %d)" % (self.id1, self.id2, self.label)


def generate_relation_pairs(relations):
    """(id1, positive id2, negative id2) for every positive x negative combination."""
    by = {}
    for r in relations:
        by.setdefault(r.id1, ([], []))[0 if r.label > 0 else 1].append(r.id2)
    out = []
    for id1, (pos, neg) in by.items():
        for p in pos:
            for n in neg:
                out.append((id1, p, n))
    return out


# ---- transformers ------------------------------------------------------------------
class TextTransformer(Preprocessing):
    def apply(self, f):
        return self.transform(f)


class Tokenizer(TextTransformer):
    def transform(self, f):
        f["tokens"] = [t for t in re.split(r"\s+", f["text"]) if t != ""]
        return f


class Normalizer(TextTransformer):
    def transform(self, f):
        f["tokens"] = [re.sub("[^a-z]", "", t.lower()) for t in f["tokens"]]
        return f


class WordIndexer(TextTransformer):
    """Unknown words map to 0 (index 0 is reserved)."""

    def __init__(self, map):  # noqa: A002 - reference name
        self.map = map

    def transform(self, f):
        f["indices"] = np.array([self.map.get(t, 0) for t in f["tokens"]], np.float32)
        return f


class SequenceShaper(TextTransformer):
    def __init__(self, len, trunc_mode="pre", pad_element=0):  # noqa: A002
        self.len, self.trunc_mode, self.pad = int(len), trunc_mode, pad_element

    def transform(self, f):
        idx = f["indices"]
        if idx.shape[0] > self.len:
            idx = idx[-self.len:] if self.trunc_mode == "pre" else idx[:self.len]
        elif idx.shape[0] < self.len:
            idx = np.concatenate([idx, np.full(self.len - idx.shape[0], self.pad, np.float32)])
        f["indices"] = idx.astype(np.float32)
        return f


class TextFeatureToSample(TextTransformer):
    def transform(self, f):
        lab = f.get("label")
        f["sample"] = (f["indices"], None if lab is None else np.array([lab], np.float32))
        return f


# ---- TextSet --------------------------------------------------------------------------
class TextSet:
    def __init__(self, features, word_index=None):
        self.features = list(features)
        self.word_index = word_index

    # construction (TextSet.scala read / readCSV / readParquet)
    @classmethod
    def read(cls, path, sc=None, min_partitions=1, distributed=False):
        """Two-level directory: one sub-folder per category (sorted names -> labels 0..n-1)."""
        feats = []
        cats = sorted(d for d in os.listdir(path) if os.path.isdir(os.path.join(path, d)))
        for label, c in enumerate(cats):
            for fn in sorted(os.listdir(os.path.join(path, c))):
                p = os.path.join(path, c, fn)
                if os.path.isfile(p):
                    with open(p, encoding="utf-8", errors="replace") as fh:
                        feats.append(TextFeature(fh.read(), label, p))
        return cls._make(feats, distributed)

    @classmethod
    def read_csv(cls, path, sc=None, min_partitions=1, distributed=False):
        """Each line ``id,text`` (the reference's readCSV format; text may contain commas)."""
        feats = []
        with open(path, encoding="utf-8") as fh:
            for row in csv.reader(fh):
                if row:
                    feats.append(TextFeature(",".join(row[1:]), None, row[0]))
        return cls._make(feats, distributed)

    @classmethod
    def read_parquet(cls, path, sc=None, distributed=False):
        """Parquet with columns ``id`` and ``text``."""
        import pyarrow.parquet as pq
        tab = pq.read_table(path).to_pydict()
        feats = [TextFeature(t, None, str(i)) for i, t in zip(tab["id"], tab["text"])]
        return cls._make(feats, distributed)

    @classmethod
    def from_texts(cls, texts, labels=None):
        return LocalTextSet([TextFeature(t, None if labels is None else labels[i], str(i))
                             for i, t in enumerate(texts)])

    @staticmethod
    def _make(feats, distributed):
        if distributed:
            from zoo.common.nncontext import get_nncontext
            ctx = get_nncontext()
            return DistributedTextSet(feats[ctx.rank::ctx.world_size])
        return LocalTextSet(feats)

    @classmethod
    def from_relation_pairs(cls, relations, corpus1, corpus2):
        """Each (id1, pos, neg) pair -> sample [2, len1+len2] (text1++pos, text1++neg), label [[1],[0]]."""
        m1 = {f["uri"]: f["indices"] for f in corpus1.features}
        m2 = {f["uri"]: f["indices"] for f in corpus2.features}
        out = []
        for id1, p, n in generate_relation_pairs(relations):
            t1, tp, tn = m1[id1], m2[p], m2[n]
            if tp.shape != tn.shape:
                raise ValueError("corpus2 contains texts with different lengths, please shape_sequence first")
            feat = np.stack([np.concatenate([t1, tp]), np.concatenate([t1, tn])]).astype(np.float32)
            f = TextFeature(None, None, id1 + p + n)
            f["sample"] = (feat, np.array([[1.0], [0.0]], np.float32))
            out.append(f)
        return LocalTextSet(out)

    @classmethod
    def from_relation_lists(cls, relations, corpus1, corpus2):
        """Per id1: every related id2 -> sample [k, len1+len2] with the relation labels [k, 1]."""
        m1 = {f["uri"]: f["indices"] for f in corpus1.features}
        m2 = {f["uri"]: f["indices"] for f in corpus2.features}
        groups = {}
        for r in relations:
            groups.setdefault(r.id1, []).append(r)
        out = []
        for id1, rs in groups.items():
            feat = np.stack([np.concatenate([m1[id1], m2[r.id2]]) for r in rs]).astype(np.float32)
            lab = np.array([[float(r.label)] for r in rs], np.float32)
            f = TextFeature(None, None, id1)
            f["sample"] = (feat, lab)
            out.append(f)
        return LocalTextSet(out)

    # API
    def is_local(self):
        return not isinstance(self, DistributedTextSet)

    def is_distributed(self):
        return isinstance(self, DistributedTextSet)

    def to_local(self):
        return LocalTextSet(self.features, self.word_index)

    def to_distributed(self, sc=None, partition_num=4):
        return DistributedTextSet(self.features, self.word_index)

    def transform(self, transformer):
        return type(self)([transformer.apply(dict(f)) for f in self.features], self.word_index)

    def __rshift__(self, t):
        return self.transform(t)

    def tokenize(self):
        return self.transform(Tokenizer())

    def normalize(self):
        return self.transform(Normalizer())

    def generate_word_index_map(self, remove_topN=0, max_words_num=-1, min_freq=1, existing_map=None):  # noqa: N803
        if remove_topN < 0:
            raise ValueError("removeTopN should be a non-negative integer")
        if not (max_words_num == -1 or max_words_num > 0):
            raise ValueError("maxWordsNum should be either -1 or a positive integer")
        if min_freq < 1:
            raise ValueError("minFreq should be a positive integer")
        tokens = [t for f in self.features for t in f["tokens"]]
        if remove_topN == 0 and max_words_num == -1 and min_freq == 1:
            words = list(dict.fromkeys(tokens))
        else:
            freq = {}
            for t in tokens:
                freq[t] = freq.get(t, 0) + 1
            items = [(w, c) for w, c in freq.items() if c >= min_freq]
            if remove_topN > 0 or max_words_num > 0:
                items.sort(key=lambda x: -x[1])  # stable, like Scala's sortBy
                words = [w for w, _ in items]
                if remove_topN > 0:
                    words = words[remove_topN:]
                if max_words_num > 0:
                    words = words[:max_words_num]
            else:
                words = [w for w, _ in items]
        index = dict(existing_map) if existing_map else {}
        nxt = max(index.values()) + 1 if index else 1
        for w in words:
            if w not in index:
                index[w] = nxt
                nxt += 1
        self.word_index = index
        return index

    def word2idx(self, remove_topN=0, max_words_num=-1, min_freq=1, existing_map=None):  # noqa: N803
        if self.word_index is None:
            self.generate_word_index_map(remove_topN, max_words_num, min_freq, existing_map)
        return self.transform(WordIndexer(self.word_index))

    def shape_sequence(self, len, trunc_mode="pre", pad_element=0):  # noqa: A002
        return self.transform(SequenceShaper(len, trunc_mode, pad_element))

    def generate_sample(self):
        return self.transform(TextFeatureToSample())

    def get_word_index(self):
        return self.word_index

    def set_word_index(self, vocab):
        self.word_index = dict(vocab)
        return self

    def save_word_index(self, path):
        with open(path, "w", encoding="utf-8") as fh:
            for w, i in self.word_index.items():
                fh.write("%s %d\n" % (w, i))

    def load_word_index(self, path):
        idx = {}
        with open(path, encoding="utf-8") as fh:
            for line in fh:
                parts = line.rstrip("\n").split(" ")
                if len(parts) == 2:
                    idx[parts[0]] = int(parts[1])
        self.word_index = idx
        return self

    def get_texts(self):
        return [f.get("text") for f in self.features]

    def get_uris(self):
        return [f.get("uri") for f in self.features]

    def get_labels(self):
        return [f.get("label", -1) for f in self.features]

    def get_predicts(self):
        return [(f.get("uri"), f.get("predict")) for f in self.features]

    def get_samples(self):
        return [f.get("sample") for f in self.features]

    def random_split(self, weights, seed=None):
        rng = np.random.default_rng(seed)
        w = np.asarray(weights, np.float64)
        w = w / w.sum()
        assign = rng.choice(len(w), size=len(self.features), p=w)
        return [type(self)([f for f, a in zip(self.features, assign) if a == k], self.word_index)
                for k in range(len(w))]

    def __len__(self):
        return len(self.features)

    def to_featureset(self, batch_size=32, shuffle=True):
        from zoo.feature.common import FeatureSet
        samples = self.get_samples()
        if any(s is None for s in samples):
            raise ValueError("call generate_sample() first")
        x = np.stack([s[0] for s in samples]).astype(np.float32)
        ys = [s[1] for s in samples]
        y = None if any(v is None for v in ys) else np.stack(ys).astype(np.float32)
        if y is not None and y.ndim == 2 and y.shape[1] == 1:
            y = y[:, 0]
        return FeatureSet.from_ndarrays(x, y, batch_size, shuffle=shuffle)


class LocalTextSet(TextSet):
    pass


class DistributedTextSet(TextSet):
    pass
