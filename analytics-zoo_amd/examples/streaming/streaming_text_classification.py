#!/usr/bin/env python3
"""Streaming text classification (pyzoo/zoo/examples/streaming/textclassification): a stream of
text lines (here a file another thread keeps appending to -- a socket / Kafka topic in
production) is cut into micro-batches; each micro-batch is tokenised with the trained word
index, padded, and classified by a TextClassifier served through InferenceModel. The model is
trained briefly on a synthetic two-topic corpus first."""
import argparse
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402

TOPICS = [["gpu", "kernel", "matrix", "wave", "memory", "tensor"], ["goal", "match", "team", "score", "league", "coach"]]


def _sentence(rng, t):
    return " ".join(rng.choice(TOPICS[t], 6))


def main(argv=None):
    ap = _common.add_common(argparse.ArgumentParser(description=__doc__.split("\n")[0]))
    ap.add_argument("--lines", type=int, default=40)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--seq-len", type=int, default=8)
    a = ap.parse_args(argv)
    import torch
    from zoo.models.textclassification import TextClassifier
    from zoo.pipeline.inference import InferenceModel
    torch.manual_seed(a.seed)
    rng = np.random.default_rng(a.seed)
    vocab = {w: i + 1 for i, w in enumerate(sorted(w for t in TOPICS for w in t))}

    def encode(lines):
        ids = np.zeros((len(lines), a.seq_len), np.float32)
        for r, s in enumerate(lines):
            toks = [vocab.get(w, 0) for w in s.split()][:a.seq_len]
            ids[r, :len(toks)] = toks
        return ids
    labels = rng.integers(0, 2, 256)
    xtr = encode([_sentence(rng, int(t)) for t in labels])
    model = TextClassifier(2, sequence_length=a.seq_len, encoder="cnn", encoder_output_dim=16,
                           vocab_size=len(vocab) + 1, embed_dim=16)
    model.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    model.fit(xtr, labels, batch_size=32, nb_epoch=a.epochs, distributed=False)
    im = InferenceModel(1).load_module(model.model if hasattr(model, "model") else model)

    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "stream.txt")
        open(path, "w").close()
        truth = []

        def producer():
            with open(path, "a") as f:
                for _ in range(a.lines):
                    t = int(rng.integers(0, 2))
                    truth.append(t)
                    f.write(_sentence(rng, t) + "\n")
                    f.flush()
                    time.sleep(0.001)
        th = threading.Thread(target=producer)
        th.start()
        preds, pos, buf = [], 0, ""
        deadline = time.time() + 60
        while len(preds) < a.lines and time.time() < deadline:
            with open(path) as f:
                f.seek(pos)
                chunk = f.read()
                pos = f.tell()
            buf += chunk
            *lines, buf = buf.split("\n")
            for i in range(0, len(lines), a.micro_batch):
                mb = lines[i:i + a.micro_batch]
                if mb:
                    p = im.predict(encode(mb))
                    preds.extend(np.asarray(p).argmax(-1).tolist())
                    print("micro-batch of %d -> %s" % (len(mb), preds[-len(mb):]))
            if not lines:
                time.sleep(0.005)
        th.join()
    acc = float(np.mean(np.asarray(preds[:len(truth)]) == np.asarray(truth[:len(preds)])))
    print("streamed %d lines, accuracy %.2f" % (len(preds), acc))
    return {"lines": len(preds), "accuracy": acc}


if __name__ == "__main__":
    main()
