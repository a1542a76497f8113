#!/usr/bin/env python3
"""Neural Collaborative Filtering (Zs/examples/recommendation/NeuralCFexample.scala,
pyzoo NCF quick start): ml-20m-shaped synthetic ratings (138,493 users x 26,744 items by
default, scale down with --users/--items), NeuralCF with the MF branch, Adam, then
recommendations for users. ``--data ratings.dat`` reads MovieLens ``u::i::r::t`` lines."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def synthetic_ratings(n, users, items, seed=0):
    rng = np.random.default_rng(seed)
    u = rng.integers(1, users + 1, n)
    i = rng.integers(1, items + 1, n)
    r = ((u * 7 + i * 3) % 5) + 1     # a learnable user-item interaction
    return np.stack([u, i], 1).astype(np.float32), r.astype(np.int64)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data", default=None)
    ap.add_argument("--users", type=int, default=138493)
    ap.add_argument("--items", type=int, default=26744)
    ap.add_argument("--n", type=int, default=200000)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--epochs", type=int, default=2)
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.models.recommendation import NeuralCF
    from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("ncf")
    if a.data:
        raw = np.loadtxt(a.data, delimiter="::", dtype=np.int64)
        x, y = raw[:, :2].astype(np.float32), raw[:, 2]
        a.users, a.items = int(raw[:, 0].max()), int(raw[:, 1].max())
    else:
        x, y = synthetic_ratings(a.n, a.users, a.items)
    m = NeuralCF(a.users, a.items, 5, user_embed=20, item_embed=20, hidden_layers=(40, 20, 10), include_mf=True,
                 mf_embed=20)
    m.compile(optimizer=Adam(lr=1e-3), loss=SparseCategoricalCrossEntropy(zero_based_label=False),
              metrics=["accuracy"])
    m.fit(x, y, batch_size=a.batch, nb_epoch=a.epochs)
    res = m.evaluate(x[:a.batch], y[:a.batch], batch_size=a.batch)
    print("train-sample metrics:", res)
    from zoo.models.recommendation.recommender import UserItemFeature
    # score 20 candidate items for two users, keep the top 3 each (Recommender.recommendForUser)
    cands = [UserItemFeature(u, it, np.array([u, it], np.float32)) for u in (1, 2) for it in range(1, 21)]
    recs = m.recommend_for_user(cands, 3)
    print("recommendations:", recs)
    return res


if __name__ == "__main__":
    main()
