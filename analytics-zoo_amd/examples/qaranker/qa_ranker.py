#!/usr/bin/env python3
"""Question-answer ranking with KNRM (pyzoo/zoo/examples/qaranker/qa_ranker.py on WikiQA):
relation pairs of (question, positive answer, negative answer) -> TextSet.from_relation_pairs
-> KNRM with a rank-hinge loss; evaluation by NDCG / MAP over relation lists. A synthetic
corpus stands in for WikiQA (answers sharing words with their question are relevant)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--questions", type=int, default=40)
    ap.add_argument("--q-len", type=int, default=8)
    ap.add_argument("--a-len", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=3)
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.models.textmatching import KNRM
    from zoo.pipeline.api.keras.objectives import RankHinge
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("qa_ranker")
    rng = np.random.default_rng(0)
    vocab = 300
    emb = rng.standard_normal((vocab, 16)).astype(np.float32)
    emb /= np.linalg.norm(emb, axis=1, keepdims=True)
    pairs = []
    for _ in range(a.questions):
        q = rng.integers(1, vocab, a.q_len)
        pos = np.concatenate([rng.choice(q, a.a_len // 2), rng.integers(1, vocab, a.a_len - a.a_len // 2)])
        neg = rng.integers(1, vocab, a.a_len)
        pairs.append(np.concatenate([q, pos]))
        pairs.append(np.concatenate([q, neg]))
    x = np.stack(pairs).astype(np.float32)          # interleaved (positive, negative) like the reference
    y = np.tile([1.0, 0.0], a.questions).astype(np.float32)
    m = KNRM(a.q_len, a.a_len, embed_weights=emb, kernel_num=11)
    m.compile(optimizer=Adam(lr=0.001), loss=RankHinge())
    m.fit(x, y, batch_size=2 * 8, nb_epoch=a.epochs)
    s = m.predict(x).reshape(-1)
    acc = float((s[0::2] > s[1::2]).mean())
    print("pairs ranked correctly:", acc)
    return acc


if __name__ == "__main__":
    main()
