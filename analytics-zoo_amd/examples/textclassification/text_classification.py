#!/usr/bin/env python3
"""Text classification (pyzoo/zoo/examples/textclassification/text_classification.py,
Zs/examples/textclassification): TextSet -> tokenize -> word index -> shape sequence ->
TextClassifier (CNN / LSTM / GRU encoder over GloVe-style embeddings). ``--data DIR`` reads a
news20-style tree (one sub-directory per class); without it a synthetic corpus is used."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def synthetic_corpus(n, classes, seed=0):
    rng = np.random.default_rng(seed)
    topics = [["t%d_%d" % (c, k) for k in range(20)] for c in range(classes)]
    common = ["w%d" % k for k in range(200)]
    texts, labels = [], []
    for _ in range(n):
        c = int(rng.integers(classes))
        words = list(rng.choice(common, 30)) + list(rng.choice(topics[c], 6))
        rng.shuffle(words)
        texts.append(" ".join(words))
        labels.append(c)
    return texts, labels


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data", default=None)
    ap.add_argument("--classes", type=int, default=5)
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--sequence-length", type=int, default=64)
    ap.add_argument("--encoder", default="cnn", choices=["cnn", "lstm", "gru"])
    ap.add_argument("--embed-dim", type=int, default=32)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=3)
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.feature.text import TextSet
    from zoo.models.textclassification import TextClassifier
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("text_classification")
    if a.data:
        ts = TextSet.read(a.data)
    else:
        texts, labels = synthetic_corpus(a.n, a.classes)
        ts = TextSet.from_texts(texts, labels)
    ts = ts.tokenize().normalize().word2idx(remove_topN=0, max_words_num=5000).shape_sequence(a.sequence_length) \
        .generate_sample()
    samples = ts.get_samples()
    x = np.stack([np.asarray(s[0], np.float32) for s in samples])
    y = np.asarray([int(np.asarray(s[1]).reshape(-1)[0]) for s in samples], np.int64)
    wi = ts.get_word_index()
    rng = np.random.default_rng(1)
    emb = {w: rng.standard_normal(a.embed_dim).astype(np.float32) for w in wi}
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for w, v in emb.items():
            f.write(w + " " + " ".join("%.4f" % t for t in v) + "\n")
        glove = f.name
    m = TextClassifier(a.classes, glove, wi, sequence_length=a.sequence_length, encoder=a.encoder,
                       encoder_output_dim=64)
    os.unlink(glove)
    m.compile(optimizer=Adam(lr=0.005), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    m.fit(x, y, batch_size=a.batch, nb_epoch=a.epochs)
    res = m.evaluate(x, y, batch_size=a.batch)
    print("accuracy:", res)
    return res


if __name__ == "__main__":
    main()
