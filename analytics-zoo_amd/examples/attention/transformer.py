#!/usr/bin/env python3
"""Text classification with the Zoo TransformerLayer (pyzoo/zoo/examples/attention/
transformer.py on IMDB): token + position ids -> TransformerLayer (native fused attention
and LayerNorm on MI355X) -> pooled output -> Dense softmax. Synthetic sequences whose label
is whether a marker token occurs (IMDB needs a download)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--vocab", type=int, default=200)
    ap.add_argument("--seq-len", type=int, default=32)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=2)
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.layers import Dense, Input, TransformerLayer
    from zoo.pipeline.api.keras.models import Model
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("transformer")
    rng = np.random.default_rng(0)
    tok = rng.integers(2, a.vocab, (a.n, a.seq_len))
    y = rng.integers(0, 2, a.n)
    tok[y == 1, rng.integers(0, a.seq_len, int((y == 1).sum()))] = 1      # marker token
    pos = np.tile(np.arange(a.seq_len), (a.n, 1))
    t_in, p_in = Input(shape=(a.seq_len,)), Input(shape=(a.seq_len,))
    tr = TransformerLayer.init(vocab=a.vocab, seq_len=a.seq_len, n_block=a.blocks, hidden_size=a.hidden,
                               n_head=a.heads, hidden_drop=0.0, attn_drop=0.0)
    pooled = tr([t_in, p_in])[1]        # (sequence output, pooled output)
    out = Dense(2, activation="softmax")(pooled)
    m = Model([t_in, p_in], out)
    m.compile(optimizer=Adam(lr=1e-3), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    m.fit([tok.astype(np.float32), pos.astype(np.float32)], y, batch_size=a.batch, nb_epoch=a.epochs)
    res = m.evaluate([tok.astype(np.float32), pos.astype(np.float32)], y, batch_size=a.batch)
    print("accuracy:", res)
    return res


if __name__ == "__main__":
    main()
