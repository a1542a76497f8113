"""TFPark text models (Py/tfpark/text/**; reference tests pyzoo/test/zoo/tfpark/
test_text_models.py and test_tfpark_estimator bert cases): CRF against brute-force
path enumeration, BERT checkpoint mapping against a numpy Google-BERT forward,
BERT estimators and the Keras taggers end to end on CPU."""
import itertools
import math

import numpy as np
import pytest
import torch

from zoo.ops.crf import crf_decode, crf_nll


def _paths_scores(e, tr, st, en, T):
    L = e.shape[-1]
    out = {}
    for path in itertools.product(range(L), repeat=T):
        s = st[path[0]] + e[0, path[0]] + en[path[-1]]
        for t in range(1, T):
            s += tr[path[t - 1], path[t]] + e[t, path[t]]
        out[path] = float(s)
    return out


def test_crf_nll_and_viterbi_vs_enumeration():
    torch.manual_seed(0)
    B, T, L = 3, 4, 3
    e = torch.randn(B, T, L)
    tr, st, en = torch.randn(L, L), torch.randn(L), torch.randn(L)
    tags = torch.randint(0, L, (B, T))
    lengths = [4, 2, 3]
    mask = torch.tensor([[1.0 if t < n else 0.0 for t in range(T)] for n in lengths])
    nll = crf_nll(e, tags, tr, mask, st, en)
    ref, best = 0.0, []
    for b in range(B):
        n = lengths[b]
        sc = _paths_scores(e[b, :n].numpy(), tr.numpy(), st.numpy(), en.numpy(), n)
        logz = math.log(sum(math.exp(v) for v in sc.values()))
        ref += logz - sc[tuple(tags[b, :n].tolist())]
        best.append(max(sc, key=sc.get))
    assert abs(float(nll) - ref / B) < 1e-4
    dec = crf_decode(e, tr, mask, st, en)
    for b in range(B):
        n = lengths[b]
        assert tuple(dec[b, :n].tolist()) == best[b]
        assert dec[b, n:].sum() == 0


def _gelu(x):
    return 0.5 * x * (1 + np.vectorize(math.erf)(x / math.sqrt(2)))


def _ln(x, g, b, eps=1e-12):
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return (x - m) / np.sqrt(v + eps) * g + b


def _numpy_google_bert(v, ids, tt, mask, H, nh, n_layers):
    """Google BERT forward (modeling.py math) straight from the TF variable dict."""
    L = ids.shape[1]
    x = v["bert/embeddings/word_embeddings"][ids] + v["bert/embeddings/token_type_embeddings"][tt] + \
        v["bert/embeddings/position_embeddings"][:L][None]
    x = _ln(x, v["bert/embeddings/LayerNorm/gamma"], v["bert/embeddings/LayerNorm/beta"])
    add = (1.0 - mask[:, None, None, :]) * -10000.0
    hd = H // nh
    for i in range(n_layers):
        p = "bert/encoder/layer_%d/" % i

        def dense(t, n):
            return t @ v[p + n + "/kernel"] + v[p + n + "/bias"]
        q, k, vv = (dense(x, "attention/self/" + n).reshape(x.shape[0], L, nh, hd).transpose(0, 2, 1, 3)
                    for n in ("query", "key", "value"))
        s = q @ k.transpose(0, 1, 3, 2) / math.sqrt(hd) + add
        s = np.exp(s - s.max(-1, keepdims=True))
        s /= s.sum(-1, keepdims=True)
        a = (s @ vv).transpose(0, 2, 1, 3).reshape(x.shape[0], L, H)
        x = _ln(dense(a, "attention/output/dense") + x, v[p + "attention/output/LayerNorm/gamma"],
                v[p + "attention/output/LayerNorm/beta"])
        m = dense(_gelu(dense(x, "intermediate/dense")), "output/dense")
        x = _ln(m + x, v[p + "output/LayerNorm/gamma"], v[p + "output/LayerNorm/beta"])
    pooled = np.tanh(x[:, 0] @ v["bert/pooler/dense/kernel"] + v["bert/pooler/dense/bias"])
    return x, pooled


def _fake_google_ckpt(H=32, nh=4, n_layers=2, inter=64, vocab=50, maxpos=16, seed=0):
    rng = np.random.default_rng(seed)
    v = {"bert/embeddings/word_embeddings": rng.normal(0, 0.5, (vocab, H)),
         "bert/embeddings/token_type_embeddings": rng.normal(0, 0.5, (2, H)),
         "bert/embeddings/position_embeddings": rng.normal(0, 0.5, (maxpos, H)),
         "bert/embeddings/LayerNorm/gamma": rng.normal(1, 0.1, H), "bert/embeddings/LayerNorm/beta": rng.normal(0, 0.1, H),
         "bert/pooler/dense/kernel": rng.normal(0, 0.2, (H, H)), "bert/pooler/dense/bias": rng.normal(0, 0.1, H)}
    for i in range(n_layers):
        p = "bert/encoder/layer_%d/" % i
        for n in ("query", "key", "value"):
            v[p + "attention/self/%s/kernel" % n] = rng.normal(0, 0.2, (H, H))
            v[p + "attention/self/%s/bias" % n] = rng.normal(0, 0.1, H)
        v[p + "attention/output/dense/kernel"] = rng.normal(0, 0.2, (H, H))
        v[p + "attention/output/dense/bias"] = rng.normal(0, 0.1, H)
        v[p + "intermediate/dense/kernel"] = rng.normal(0, 0.2, (H, inter))
        v[p + "intermediate/dense/bias"] = rng.normal(0, 0.1, inter)
        v[p + "output/dense/kernel"] = rng.normal(0, 0.2, (inter, H))
        v[p + "output/dense/bias"] = rng.normal(0, 0.1, H)
        for ln in ("attention/output/LayerNorm", "output/LayerNorm"):
            v[p + ln + "/gamma"] = rng.normal(1, 0.1, H)
            v[p + ln + "/beta"] = rng.normal(0, 0.1, H)
    return {k: np.asarray(a, np.float32) for k, a in v.items()}


def _cfg(**kw):
    from zoo.tfpark.text.estimator import BertConfig
    d = dict(vocab_size=50, hidden_size=32, num_hidden_layers=2, num_attention_heads=4, intermediate_size=64,
             max_position_embeddings=16, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    d.update(kw)
    return BertConfig(**d)


def test_google_bert_checkpoint_matches_numpy_reference(monkeypatch):
    from zoo.pipeline.api.net import tf_graph
    from zoo.tfpark.text.estimator import BertEncoder, load_bert_checkpoint
    v = _fake_google_ckpt()
    monkeypatch.setattr(tf_graph, "read_tensor_bundle", lambda prefix: v)
    enc = BertEncoder(_cfg())
    used = load_bert_checkpoint(enc.bert, "unused")
    assert len(used) == len(v)
    enc.eval()
    rng = np.random.default_rng(1)
    ids = rng.integers(0, 50, (2, 10))
    tt = rng.integers(0, 2, (2, 10))
    mask = np.ones((2, 10), np.float32)
    mask[1, 7:] = 0
    with torch.no_grad():
        seq, pooled = enc({"input_ids": torch.from_numpy(ids), "token_type_ids": torch.from_numpy(tt),
                           "input_mask": torch.from_numpy(mask)})
    rs, rp = _numpy_google_bert(v, ids, tt, mask, 32, 4, 2)
    np.testing.assert_allclose(seq.numpy(), rs, atol=2e-4, rtol=1e-3)
    np.testing.assert_allclose(pooled.numpy(), rp, atol=2e-4, rtol=1e-3)


def _bert_rows(n, L, label_fn):
    rng = np.random.default_rng(0)
    rows = []
    for _ in range(n):
        ids = rng.integers(1, 50, L)
        feats = {"input_ids": ids, "input_mask": np.ones(L, np.int64), "token_type_ids": np.zeros(L, np.int64)}
        rows.append((feats, label_fn(ids)))
    return rows


def test_bert_classifier_learns_and_predicts():
    from zoo.tfpark.text.estimator import BERTClassifier, bert_input_fn
    from zoo.pipeline.api.keras.optimizers import Adam
    torch.manual_seed(0)
    rows = _bert_rows(64, 8, lambda ids: int(ids[0] > 25))
    est = BERTClassifier(2, _cfg(), optimizer=Adam(lr=2e-3))
    fn = bert_input_fn(rows, 8, 16)
    before = est.evaluate(fn)["loss"]
    est.train(fn, steps=60)
    after = est.evaluate(fn)
    assert after["loss"] < before and after["acc"] > 0.8, (before, after)
    probs = est.predict(bert_input_fn([r[0] for r in rows[:5]], 8, 4))
    assert probs.shape == (5, 2) and np.allclose(probs.sum(1), 1, atol=1e-5)


def test_bert_ner_and_squad_heads():
    from zoo.tfpark.text.estimator import BERTNER, BERTSQuAD, bert_input_fn
    torch.manual_seed(0)
    ner = BERTNER(5, _cfg())
    rows = _bert_rows(16, 8, lambda ids: (ids % 5).astype(np.int64))
    ner.train(bert_input_fn(rows, 8, 8), steps=2)
    pred = ner.predict(bert_input_fn([r[0] for r in rows], 8, 8))
    assert pred.shape == (16, 8) and pred.max() < 5
    sq = BERTSQuAD(_cfg())
    srows = _bert_rows(16, 8, lambda ids: {"start_positions": np.int64(1), "end_positions": np.int64(3)})
    sq.train(bert_input_fn(srows, 8, 8), steps=2)
    out = sq.predict(bert_input_fn([r[0] for r in srows], 8, 8))
    assert out["start_logits"].shape == (16, 8) and out["end_logits"].shape == (16, 8)


def _tag_data(n=48, T=6, W=4):
    rng = np.random.default_rng(0)
    words = rng.integers(1, 30, (n, T))
    chars = rng.integers(1, 20, (n, T, W))
    tags = (words % 3).astype(np.int64)
    return words, chars, tags


def test_ner_fit_predict_save_load(tmp_path):
    from zoo.tfpark.text.keras import NER
    torch.manual_seed(0)
    words, chars, tags = _tag_data()
    from zoo.pipeline.api.keras.optimizers import Adam
    m = NER(3, 30, 20, word_length=4, word_emb_dim=16, char_emb_dim=8, tagger_lstm_dim=16, dropout=0.0,
            optimizer=Adam(lr=1e-2))
    hist = m.fit([words, chars], np.eye(3)[tags], batch_size=16, epochs=20)
    assert hist[-1] < hist[0]
    p = m.predict([words, chars])
    assert p.shape == (48, 6, 3)
    assert (p.argmax(-1) == tags).mean() > 0.8
    path = str(tmp_path / "ner.model")
    m.save_model(path)
    m2 = NER.load_model(path)
    np.testing.assert_array_equal(m2.predict([words, chars]), p)


def test_intent_entity_and_sequence_tagger():
    from zoo.tfpark.text.keras import IntentEntity, SequenceTagger
    torch.manual_seed(0)
    words, chars, tags = _tag_data(32)
    intents = (words[:, 0] % 2).astype(np.int64)
    ie = IntentEntity(2, 3, 30, 20, word_length=4, word_emb_dim=16, char_emb_dim=8, char_lstm_dim=8,
                      tagger_lstm_dim=16)
    ie.fit([words, chars], [intents, tags], batch_size=16, epochs=2)
    pi, ps = ie.predict([words, chars])
    assert pi.shape == (32, 2) and ps.shape == (32, 6, 3)
    st = SequenceTagger(4, 3, 30, feature_size=16, classifier="crf")
    st.fit(words, [words % 4, tags], batch_size=16, epochs=2)
    pp, pc = st.predict(words)
    assert pp.shape == (32, 6, 4) and pc.shape == (32, 6, 3)
    assert np.isfinite(st.evaluate(words, [words % 4, tags])["loss"])


def test_tf_predictor_over_dataset():
    from zoo.tfpark import TFDataset
    from zoo.tfpark.tf_predictor import TFPredictor
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    m = Sequential()
    m.add(Dense(3, input_shape=(4,)))
    x = np.random.rand(10, 4).astype(np.float32)
    ds = TFDataset.from_ndarrays(x, batch_per_thread=4)
    out = TFPredictor.from_keras(m, ds).predict()
    with torch.no_grad():
        ref = m(torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_bert_encoder_gpu_matches_numpy_reference(gpu, monkeypatch):
    """The checkpoint-loaded encoder on the native GPU path (MFMA GEMMs, fused
    attention, native LayerNorm; bf16 compute) against the fp32 numpy BERT."""
    from zoo.pipeline.api.net import tf_graph
    from zoo.tfpark.text.estimator import BertEncoder, load_bert_checkpoint
    v = _fake_google_ckpt(H=64, nh=4, inter=128, vocab=50, maxpos=32)
    monkeypatch.setattr(tf_graph, "read_tensor_bundle", lambda prefix: v)
    enc = BertEncoder(_cfg(hidden_size=64, intermediate_size=128, max_position_embeddings=32))
    load_bert_checkpoint(enc.bert, "unused")
    enc = enc.to(gpu).eval()
    rng = np.random.default_rng(2)
    ids = rng.integers(0, 50, (4, 32))
    tt = rng.integers(0, 2, (4, 32))
    mask = np.ones((4, 32), np.float32)
    mask[2, 20:] = 0
    with torch.no_grad():
        seq, pooled = enc({"input_ids": torch.from_numpy(ids).to(gpu), "token_type_ids": torch.from_numpy(tt).to(gpu),
                           "input_mask": torch.from_numpy(mask).to(gpu)})
    rs, rp = _numpy_google_bert(v, ids, tt, mask, 64, 4, 2)
    err = np.abs(seq.float().cpu().numpy() - rs).max() / np.abs(rs).max()
    assert err < 5e-2, err
    assert np.abs(pooled.float().cpu().numpy() - rp).max() < 5e-2


@pytest.mark.gpu
def test_bert_classifier_and_ner_train_on_gpu(gpu):
    from zoo.tfpark.text.estimator import BERTClassifier, bert_input_fn
    from zoo.tfpark.text.keras import NER
    from zoo.pipeline.api.keras.optimizers import Adam
    torch.manual_seed(0)
    rows = _bert_rows(64, 16, lambda ids: int(ids[0] > 25))
    est = BERTClassifier(2, _cfg(hidden_size=64, intermediate_size=128), optimizer=Adam(lr=2e-3))
    fn = bert_input_fn(rows, 16, 16)
    before = est.evaluate(fn)["loss"]
    est.train(fn, steps=60)
    after = est.evaluate(fn)
    assert after["loss"] < before and after["acc"] > 0.8, (before, after)
    words, chars, tags = _tag_data()
    m = NER(3, 30, 20, word_length=4, word_emb_dim=16, char_emb_dim=8, tagger_lstm_dim=16, dropout=0.0,
            optimizer=Adam(lr=1e-2))
    hist = m.fit([words, chars], np.eye(3)[tags], batch_size=16, epochs=5)
    assert np.isfinite(hist[-1]) and hist[-1] < hist[0]


def test_tfdataset_from_tfrecord_and_iterable(tmp_path):
    """TFDataset.from_tfrecord_file (tf.train.Example codec over TFRecord framing) and
    from_tf_data_dataset (any iterable of unbatched elements)."""
    from zoo.tfpark.tf_dataset import TFDataset, encode_example, parse_example, write_tfrecord
    rng = np.random.RandomState(0)
    xs, ys = rng.randn(10, 3).astype(np.float32), rng.randint(0, 5, 10)
    recs = [encode_example({"a": xs[i, :2], "b": xs[i, 2:], "label": [ys[i]], "name": "r%d" % i,
                            "neg": [-3, 7]}) for i in range(10)]
    ex = parse_example(recs[4])
    np.testing.assert_allclose(ex["a"], xs[4, :2])
    assert ex["label"].dtype == np.int64 and ex["label"][0] == ys[4]
    assert list(ex["neg"]) == [-3, 7] and ex["name"][0] == b"r4"
    p = str(tmp_path / "d.tfrecord")
    write_tfrecord(p, recs)
    ds = TFDataset.from_tfrecord_file(p, batch_size=5, feature_keys=["a", "b"], label_key="label")
    got_x, got_y = [], []
    for b in ds.get_training_data().data(train=False):
        got_x.append(np.asarray(b[0]))
        got_y.append(np.asarray(b[1]))
    np.testing.assert_allclose(np.concatenate(got_x), xs, rtol=1e-6)
    np.testing.assert_array_equal(np.concatenate(got_y).reshape(-1), ys)
    ds2 = TFDataset.from_tf_data_dataset([(xs[i], ys[i]) for i in range(10)], batch_size=4)
    n = sum(np.asarray(b[0]).shape[0] for b in ds2.get_training_data().data(train=False))
    assert n == 10
