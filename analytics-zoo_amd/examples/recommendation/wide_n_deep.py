#!/usr/bin/env python3
"""Wide & Deep (Zs/examples/recommendation/WideAndDeepExample.scala, pyzoo
wide_n_deep notebook): census-style columns in a pandas DataFrame, hashed wide cross
columns (SparseEmbedding bag on the native embedding-bag kernel), indicator + embedding +
continuous deep columns, trained through the Keras API."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--model-type", default="wide_n_deep", choices=["wide", "deep", "wide_n_deep"])
    a = ap.parse_args(argv)
    import pandas as pd
    from zoo.common.nncontext import init_nncontext
    from zoo.models.recommendation import ColumnFeatureInfo, WideAndDeep
    from zoo.models.recommendation.utils import row_to_sample, samples_to_arrays
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("wide_n_deep")
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"gender": rng.integers(0, 2, a.n), "age": rng.integers(0, 7, a.n),
                       "occupation": rng.integers(0, 21, a.n), "age_gender": rng.integers(0, 100, a.n),
                       "userId": rng.integers(1, 1000, a.n), "itemId": rng.integers(1, 500, a.n),
                       "hours": rng.random(a.n)})
    df["label"] = ((df["gender"] + df["age"] + df["occupation"]) % 2) + 1
    ci = ColumnFeatureInfo(wide_base_cols=["gender", "age"], wide_base_dims=[2, 7], wide_cross_cols=["age_gender"],
                           wide_cross_dims=[100], indicator_cols=["occupation"], indicator_dims=[21],
                           embed_cols=["userId", "itemId"], embed_in_dims=[1000, 500], embed_out_dims=[16, 16],
                           continuous_cols=["hours"])
    samples = [row_to_sample(r, ci, a.model_type) for _, r in df.iterrows()]
    xs, y = samples_to_arrays(samples)
    m = WideAndDeep(2, ci, model_type=a.model_type, hidden_layers=(40, 20, 10))
    m.compile(optimizer=Adam(lr=0.005), loss=ClassNLLCriterion(log_prob_as_input=False, zero_based_label=False))
    m.fit(xs if len(xs) > 1 else xs[0], y, batch_size=a.batch, nb_epoch=a.epochs)
    res = m.evaluate(xs if len(xs) > 1 else xs[0], y, batch_size=a.batch)
    print("loss:", res)
    return res


if __name__ == "__main__":
    main()
