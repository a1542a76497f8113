"""Built-in models (WideAndDeepSpec, SessionRecommenderSpec, TextClassifierSpec,
KNRMSpec, Seq2seqSpec, AnomalyDetectorSpec analogues): shapes, a few training
steps that reduce the loss, save/load, and model-specific helpers."""
import numpy as np
import pandas as pd
import pytest
import torch

from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _fit_reduces(model, x, y, loss, epochs=8, lr=0.01, bs=16):
    from zoo.pipeline.api.keras.optimizers import Adam
    model.compile(optimizer=Adam(lr=lr), loss=loss)
    before = model.evaluate(x, y, batch_size=bs)[0]
    model.fit(x, y, batch_size=bs, nb_epoch=epochs)
    after = model.evaluate(x, y, batch_size=bs)[0]
    assert after < before, (before, after)
    return after


def test_wide_and_deep_all_modes():
    from zoo.models.recommendation import ColumnFeatureInfo, WideAndDeep
    from zoo.models.recommendation.utils import row_to_sample, samples_to_arrays
    rng = np.random.default_rng(0)
    n = 96
    df = pd.DataFrame({"gender": rng.integers(0, 2, n), "age": rng.integers(0, 5, n), "occ": rng.integers(0, 7, n),
                       "cross": rng.integers(0, 20, n), "userId": rng.integers(1, 30, n),
                       "itemId": rng.integers(1, 40, n), "hours": rng.random(n)})
    df["label"] = ((df["gender"] + df["age"]) % 2) + 1
    ci = ColumnFeatureInfo(wide_base_cols=["gender", "age"], wide_base_dims=[2, 5], wide_cross_cols=["cross"],
                           wide_cross_dims=[20], indicator_cols=["occ"], indicator_dims=[7],
                           embed_cols=["userId", "itemId"], embed_in_dims=[30, 40], embed_out_dims=[8, 8],
                           continuous_cols=["hours"])
    for mt in ("wide", "deep", "wide_n_deep"):
        samples = [row_to_sample(r, ci, mt) for _, r in df.iterrows()]
        xs, y = samples_to_arrays(samples)
        m = WideAndDeep(2, ci, model_type=mt, hidden_layers=(16, 8))
        out = m.predict(xs if len(xs) > 1 else xs[0])
        assert out.shape == (n, 2) and np.allclose(out.sum(1), 1, atol=1e-5)
        from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
        _fit_reduces(m, xs if len(xs) > 1 else xs[0], y,
                     ClassNLLCriterion(log_prob_as_input=False, zero_based_label=False), epochs=10)


def test_session_recommender_with_history():
    from zoo.models.recommendation import SessionRecommender
    rng = np.random.default_rng(1)
    sess = rng.integers(1, 20, (64, 5)).astype(np.float32)
    hist = rng.integers(1, 20, (64, 4)).astype(np.float32)
    y = (sess[:, -1] - 1).astype(np.int64)  # next item = last item (learnable)
    m = SessionRecommender(20, 8, rnn_hidden_layers=(16, 16), session_length=5, include_history=True,
                           mlp_hidden_layers=(16,), history_length=4)
    assert m.predict([sess, hist]).shape == (64, 20)
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    _fit_reduces(m, [sess, hist], y, ClassNLLCriterion(log_prob_as_input=False), epochs=10, lr=0.02)
    recs = m.recommend_for_session([sess[:2], hist[:2]], 3, zero_based_label=False)
    assert len(recs) == 2 and len(recs[0]) == 3 and all(1 <= i <= 20 for i, _ in recs[0])


@pytest.mark.parametrize("encoder", ["cnn", "lstm", "gru"])
def test_text_classifier(tmp_path, encoder):
    from zoo.models.textclassification import TextClassifier
    glove = tmp_path / "glove.txt"
    glove.write_text("\n".join("w%d %s" % (i, " ".join("%.3f" % v for v in np.random.rand(6))) for i in range(30)))
    wi = {"w%d" % i: i + 1 for i in range(30)}
    m = TextClassifier(3, str(glove), wi, sequence_length=12, encoder=encoder, encoder_output_dim=16)
    x = np.random.default_rng(2).integers(0, 31, (48, 12)).astype(np.float32)
    y = (x[:, 0] % 3).astype(np.int64)
    assert m.predict(x).shape == (48, 3)
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    _fit_reduces(m, x, y, ClassNLLCriterion(log_prob_as_input=False), epochs=6, lr=0.01)


def test_knrm_kernel_pooling_matches_reference_formula():
    from zoo.models.textmatching import KNRM
    rng = np.random.default_rng(3)
    emb = rng.standard_normal((25, 8)).astype(np.float32)
    emb /= np.linalg.norm(emb, axis=1, keepdims=True)
    m = KNRM(4, 6, embed_weights=emb, kernel_num=5, target_mode="classification")
    x = rng.integers(0, 25, (3, 10)).astype(np.float32)
    out = m.predict(x)
    assert out.shape == (3, 1) and ((out > 0) & (out < 1)).all()
    # kernel features vs a loop over the reference's per-kernel formula (KNRM.scala)
    kp = [l for l in m.flattened_layers() if type(l).__name__ == "KernelPooling"][0]
    e = torch.from_numpy(emb[x.astype(np.int64)])
    phi = kp.call(e).numpy()
    q, d = emb[x[:, :4].astype(np.int64)], emb[x[:, 4:].astype(np.int64)]
    mm = np.einsum("bik,bjk->bij", q, d)
    for i in range(5):
        mu = 1.0 / 4 + 2.0 * i / 4 - 1.0
        s = 0.1
        if mu > 1.0:
            mu, s = 1.0, 0.001
        ref = np.log(np.exp(-0.5 * (mm - mu) ** 2 / s / s).sum(2) + 1.0).sum(1)
        assert np.allclose(phi[:, i], ref, rtol=1e-4, atol=1e-4)


def test_seq2seq_train_and_infer():
    from zoo.models.seq2seq import Bridge, RNNDecoder, RNNEncoder, Seq2seq
    from zoo.pipeline.api.keras.layers import Dense, TimeDistributed
    torch.manual_seed(0)
    enc = RNNEncoder.initialize("lstm", 2, 16)
    dec = RNNDecoder.initialize("lstm", 2, 16)
    m = Seq2seq(enc, dec, input_shape=(6, 3), output_shape=(5, 3), bridge=Bridge.initialize("dense", 16),
                generator=TimeDistributed(Dense(3)))
    rng = np.random.default_rng(4)
    src = rng.standard_normal((32, 6, 3)).astype(np.float32)
    dec_in = rng.standard_normal((32, 5, 3)).astype(np.float32)
    tgt = np.repeat(src[:, :1], 5, 1)  # copy the first source step
    out = m.predict([src, dec_in])
    assert out.shape == (32, 5, 3)
    _fit_reduces(m, [src, dec_in], tgt, "mse", epochs=15, lr=0.01)
    res = m.infer(src[0], np.zeros(3, np.float32), max_seq_len=4)
    assert res.shape == (1, 5, 3)


def test_anomaly_detector_unroll_and_detect():
    from zoo.models.anomalydetection import AnomalyDetector
    t = np.sin(np.arange(200) / 5.0).astype(np.float32)
    t[150] += 3.0
    un = AnomalyDetector.unroll(t.reshape(-1, 1), 10)
    assert len(un) == 190 and un[0].feature.shape == (10, 1) and un[0].label == pytest.approx(t[10])
    x, y, idx = AnomalyDetector.to_arrays(un)
    m = AnomalyDetector((10, 1), hidden_layers=(8, 8), dropouts=(0.0, 0.0))
    _fit_reduces(m, x, y, "mse", epochs=5, lr=0.01, bs=32)
    pred = m.predict(x).reshape(-1)
    flags = AnomalyDetector.detect_anomalies(y, pred, anomaly_size=3)
    assert sum(f[2] for f in flags) >= 3
    assert flags[140][2]  # the spike (index 150 = window 140's label)
