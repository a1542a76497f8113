"""AutoML / Zouwu behaviour mirrored from the reference test-suite on synthetic series
(pyzoo/test/zoo/automl/{feature,model,pipeline,regression}/*, pyzoo/test/zoo/zouwu/*):
feature transformer naming / checks / rolling / NaN masking / list inputs / post-processing /
save-restore bundles, the three models' fit_eval / save / restore / MC-dropout uncertainty,
pipeline save / load / incremental fit / multi-step evaluate, recipe look-back validation, the
Zouwu forecasters (MTNet long/short preprocessing, uncertainty, data-parallel fit over a gloo
process group) and AutoTS."""
import os
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest

from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


SEL = ["IS_AWAKE(datetime)", "IS_BUSY_HOURS(datetime)", "HOUR(datetime)"]


def _df(n, cols=("values",), start="1/1/2019", seed=0):
    rng = np.random.default_rng(seed)
    d = {"datetime": pd.date_range(start, periods=n)}
    for c in cols:
        d[c] = rng.standard_normal(n)
    return pd.DataFrame(d)


def _ft(**kw):
    from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
    base = dict(future_seq_len=1, dt_col="datetime", target_col="values", drop_missing=True)
    base.update(kw)
    return TimeSequenceFeatureTransformer(**base)


# ------------------------------------------------------------------ feature transformer
def test_feature_list_names():
    df = _df(8, ("values", "A", "B"))
    assert set(_ft(extra_features_col=["A", "B"]).get_feature_list(df)) == {
        "IS_AWAKE(datetime)", "IS_BUSY_HOURS(datetime)", "HOUR(datetime)", "DAY(datetime)", "IS_WEEKEND(datetime)",
        "WEEKDAY(datetime)", "MONTH(datetime)", "A", "B"}


def test_fit_transform_shapes_scaling_and_lists():
    df = _df(8, ("values", "A", "B"))
    cfg = {"selected_features": SEL + ["A"], "past_seq_len": 2}
    x, y = _ft().fit_transform(df, **cfg)
    assert x.shape == (6, 2, 5) and y.shape == (6, 1)
    # standard-scaled target (the first column) over the whole frame has zero mean
    assert abs(np.mean(np.concatenate([x[0, :, 0], y[:, 0]]))) < 1e-5
    xs, ys = _ft().fit_transform([df] * 3, **cfg)
    assert xs.shape == (18, 2, 5) and ys.shape == (18, 1)
    np.testing.assert_array_almost_equal(xs[:6], xs[6:12])


def test_input_checks():
    ft = _ft()
    cfg = {"selected_features": SEL, "past_seq_len": 2}
    df = _df(8)
    bad = df.assign(datetime=df["datetime"].dt.strftime("%m/%d/%Y"))
    with pytest.raises(ValueError, match="np.datetime64"):
        ft.fit_transform(bad, **cfg)
    nat = df.copy()
    nat.loc[1, "datetime"] = None
    with pytest.raises(ValueError, match=r".* datetime .*"):
        ft.fit_transform(nat, **cfg)
    with pytest.raises(ValueError, match=r".* current .*"):
        ft.fit_transform(_df(8, start="1/1/2119"), **cfg)
    gap = df.drop(index=3).reset_index(drop=True)
    with pytest.raises(ValueError, match="not uniform"):
        ft.fit_transform(gap, **cfg)


def test_input_length_checks_with_split():
    from zoo.automl.common.util import split_input_df
    df = _df(100)
    train_df, val_df, test_df = split_input_df(df, ts_col="datetime", overlap=10, val_split_ratio=0.1,
                                               test_split_ratio=0.1)
    assert len(train_df) == 80 and len(val_df) == 20 and len(test_df) == 20
    ft = _ft()
    cfg = {"selected_features": SEL, "past_seq_len": 20}
    with pytest.raises(ValueError, match="past sequence length"):
        ft.fit_transform(train_df[:20], **cfg)
    ft.fit_transform(train_df, **cfg)
    with pytest.raises(ValueError, match="past sequence length"):
        ft.transform(val_df, is_train=True)
    with pytest.raises(ValueError, match="past sequence length"):
        ft.transform(test_df[:-1], is_train=False)
    x, y = ft.transform(test_df, is_train=False)
    assert len(x) == 1 and y is None


def test_nan_windows_dropped():
    df = _df(8)
    df.loc[2, "values"] = None
    x, y = _ft().fit_transform(df, selected_features=SEL, past_seq_len=2)
    assert x.shape == (3, 2, 4) and y.shape == (3, 1)     # mask_x & mask_y = [0, 0, 0, 1, 1, 1]


def test_transform_val_and_test_lists():
    df = _df(16, ("values", "feature_1"))
    cfg = {"selected_features": SEL + ["feature_1"], "past_seq_len": 2}
    ft = _ft(extra_features_col="feature_1")
    ft.fit_transform([df[:10]] * 3, **cfg)
    vx, vy = ft.transform([df[10:]] * 3, is_train=True)
    assert vx.shape == (12, 2, 5) and vy.shape == (12, 1)
    tx, ty = ft.transform([df[10:]] * 3, is_train=False)
    assert tx.shape == (15, 2, 5) and ty is None


def test_save_restore_and_post_processing():
    from zoo.automl.common.util import restore, save
    df = _df(8, start="1/1/2019")
    ft = _ft(future_seq_len=1)
    cfg = {"selected_features": SEL, "past_seq_len": 2}
    x, y = ft.fit_transform(df, **cfg)
    truth, pred = ft.post_processing(df, y, is_train=True)
    np.testing.assert_array_almost_equal(truth, pred, decimal=5)
    np.testing.assert_array_almost_equal(truth, df[2:][["values"]].values, decimal=5)
    d = tempfile.mkdtemp()
    try:
        save(d, feature_transformers=ft)
        from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
        ft2 = TimeSequenceFeatureTransformer()
        restore(d, feature_transformers=ft2, config=cfg)
        assert (ft2.future_seq_len, ft2.dt_col, ft2.target_col, ft2.extra_features_col, ft2.drop_missing) == \
            (1, "datetime", "values", None, True)
        tx, _ = ft2.transform(df[:-1], is_train=False)
        np.testing.assert_array_almost_equal(tx, x, decimal=5)
        out = ft2.post_processing(df[:-1], y, is_train=False)
        target = df[2:].reset_index(drop=True)
        assert out["datetime"].equals(target["datetime"])
        np.testing.assert_array_almost_equal(out["values"].values, target["values"].values, decimal=5)
        outs = ft2.post_processing([df[:-1]] * 2, np.concatenate([y, y]), is_train=False)
        assert len(outs) == 2 and outs[0].equals(outs[1])
    finally:
        shutil.rmtree(d)


def test_post_processing_multi_step():
    df = _df(8)
    ft = _ft(future_seq_len=2)
    x, y = ft.fit_transform(df, selected_features=SEL, past_seq_len=2)
    out = ft.post_processing(df[:-2], y, is_train=False)
    assert out.shape == (8 - 2 - 2 + 1, 3)
    target = df[2:].reset_index(drop=True)
    np.testing.assert_array_almost_equal(out[["values_0", "values_1"]].values,
                                         ft._roll_test(target["values"], 2), decimal=5)
    assert out["datetime"].equals(target[:-1]["datetime"])


# ------------------------------------------------------------------ models
def _rolled(ft, n, past, future=1, feat=4, seed=0):
    data = pd.DataFrame(np.random.default_rng(seed).standard_normal((n, feat)))
    return ft._roll_train(data, past, future)


@pytest.mark.parametrize("kind", ["MTNet", "Seq2seq", "LSTM"])
def test_model_fit_eval_save_restore_uncertainty(kind, tmp_path):
    from zoo.automl.common.util import restore, save
    from zoo.automl.model import LSTMSeq2Seq, MTNetKeras, VanillaLSTM
    ft = _ft()
    long_num, time_step = 6, 2
    past = (long_num + 1) * time_step
    future = 1 if kind != "Seq2seq" else 2
    x, y = _rolled(ft, 64, past, future)
    vx, vy = _rolled(ft, 16, past, future, seed=1)
    tx = ft._roll_test(pd.DataFrame(np.random.default_rng(2).standard_normal((16, 4))), past)
    cls = {"MTNet": MTNetKeras, "Seq2seq": LSTMSeq2Seq, "LSTM": VanillaLSTM}[kind]
    cfg = {"epochs": 1}
    if kind == "MTNet":
        cfg.update(long_num=long_num, time_step=time_step, ar_window=2, cnn_height=2)
    if kind == "Seq2seq":
        cfg.update(latent_dim=16)
    m = cls(check_optional_config=False, future_seq_len=future)
    m.fit_eval(x, y, validation_data=(vx, vy), mc=True, **cfg)
    m.evaluate(vx, vy)
    pred = m.predict(tx)
    assert pred.shape == (tx.shape[0], y.shape[1])
    d = str(tmp_path / "m")
    save(d, model=m)
    m2 = cls(check_optional_config=False, future_seq_len=future)
    restore(d, model=m2, config=cfg)
    np.testing.assert_array_almost_equal(pred, m2.predict(tx), decimal=4)
    m2.fit_eval(x, y, epochs=1)
    mean, unc = m.predict_with_uncertainty(tx, n_iter=3)
    assert mean.shape == pred.shape and unc.shape == pred.shape and np.any(unc)


# ------------------------------------------------------------------ pipeline / predictor
def _tsp(future, target="values"):
    from zoo.automl.regression.time_sequence_predictor import TimeSequencePredictor
    return TimeSequencePredictor(dt_col="datetime", target_col=target, future_seq_len=future, extra_features_col=None)


def test_pipeline_save_load_fit_future_1(tmp_path):
    from zoo.automl.model.time_sequence import TimeSequenceModel
    from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
    from zoo.automl.pipeline.time_sequence import load_ts_pipeline
    train_df, test_df = _df(120, seed=1), _df(25, seed=2)
    ppl = _tsp(1).fit(train_df, test_df)
    y_pred = ppl.predict(test_df)
    mse, rs = ppl.evaluate(test_df, metrics=["mse", "r2"])
    f = str(tmp_path / "my.ppl")
    ppl.save(f)
    assert os.path.isfile(f)
    new = load_ts_pipeline(f)
    assert new.config is not None and isinstance(new.feature_transformers, TimeSequenceFeatureTransformer)
    assert isinstance(new.model, TimeSequenceModel)
    new.describe()
    np.testing.assert_array_almost_equal(y_pred["values"].values, new.predict(test_df)["values"].values, decimal=4)
    new.fit(train_df, epoch_num=1)
    assert len(new.evaluate(test_df, metrics=["mse", "r2"])) == 2


def test_pipeline_multi_step_evaluate_matches_predict():
    from zoo.automl.common.metrics import Evaluator
    from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
    future = 3
    train_df, test_df = _df(120, seed=3), _df(25, seed=4)
    ppl = _tsp(future).fit(train_df, test_df)
    mse, rs = ppl.evaluate(test_df, metrics=["mse", "r2"])
    assert len(mse) == future and len(rs) == future
    assert ppl.predict(test_df).shape == (25 - 2 + 1, future + 1)
    pdf = ppl.predict(test_df[:-future])
    pv = pdf[["values_%d" % i for i in range(future)]].values
    yv = TimeSequenceFeatureTransformer()._roll_test(test_df[2:]["values"], future)
    np.testing.assert_array_almost_equal(Evaluator.evaluate("mse", yv, pv), mse, decimal=4)


def test_predict_df_list():
    train_df, test_df = _df(100, seed=5), _df(22, seed=6)
    ppl = _tsp(2).fit([train_df] * 2, [test_df] * 2)
    y = ppl.predict([test_df] * 2)
    assert len(y) == 2 and y[0].shape == (22 - 2 + 1, 3)
    pd.testing.assert_frame_equal(y[0], y[1])


def test_look_back_validation():
    from zoo.automl.config.recipe import RandomRecipe
    RandomRecipe(look_back=(1, 2))
    with pytest.raises(ValueError, match="max look back value"):
        RandomRecipe(look_back=(0, 1))
    with pytest.raises(ValueError, match="look back value should not be smaller than 2"):
        RandomRecipe(look_back=1)
    for bad in (None, "a", 2.5, (2.5, 3)):
        with pytest.raises(ValueError, match="look_back should be either"):
            RandomRecipe(look_back=bad)


def test_fit_with_fixed_configs_and_uncertainty():
    from zoo.automl.pipeline.time_sequence import TimeSequencePipeline
    train_df, test_df = _df(80, seed=7), _df(20, seed=8)
    ppl = TimeSequencePipeline(name="fixed")
    defaults = ppl.get_default_configs()
    assert defaults["past_seq_len"] == 2 and defaults["future_seq_len"] == 1
    ppl.fit_with_fixed_configs(train_df, test_df, mc=True, target_col="values", epochs=1, past_seq_len=3)
    out, unc = ppl.predict_with_uncertainty(test_df, n_iter=3)
    assert len(out) == 20 - 3 + 1 and unc.shape[0] == len(out)


# ------------------------------------------------------------------ zouwu
def _zouwu_data():
    ft = _ft()
    past = (6 + 1) * 2
    x, y = _rolled(ft, 64, past)
    vx, vy = _rolled(ft, 16, past, seed=1)
    tx = ft._roll_test(pd.DataFrame(np.random.default_rng(2).standard_normal((16, 4))), past)
    return x, y, vx, vy, tx


def test_forecast_lstm_and_mtnet():
    from zoo.zouwu.model.forecast import LSTMForecaster, MTNetForecaster
    x, y, vx, vy, tx = _zouwu_data()
    m = LSTMForecaster(horizon=1, feature_dim=x.shape[-1])
    m.fit(x, y, validation_data=(vx, vy), batch_size=8, distributed=False)
    m.evaluate(vx, vy)
    assert m.predict(tx).shape == (len(tx), 1)
    mt = MTNetForecaster(horizon=1, feature_dim=x.shape[-1], lb_long_steps=6, lb_long_stepsize=2, uncertainty=True)
    xl, xs = mt.preprocess_input(x)
    assert xl.shape == (len(x), 6, 2, 4) and xs.shape == (len(x), 2, 4)
    vl, vs = mt.preprocess_input(vx)
    tl, ts = mt.preprocess_input(tx)
    mt.fit([xl, xs], y, validation_data=([vl, vs], vy), batch_size=32, distributed=False)
    mt.evaluate([vl, vs], vy)
    assert mt.predict([tl, ts]).shape == (len(tx), 1)
    mean, std = mt.predict_with_uncertainty([tl, ts], n_iter=3)
    assert mean.shape == std.shape == (len(tx), 1) and np.any(std)


def _dist_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        from zoo.zouwu.model.forecast import LSTMForecaster
        rng = np.random.default_rng(0)
        x = rng.standard_normal((64, 6, 2)).astype(np.float32)
        y = (x[:, -1, :1] * 0.5).astype(np.float32)
        f = LSTMForecaster(horizon=1, feature_dim=2, lr=0.01)
        before = f.evaluate(x, y)[0]
        f.fit(x, y, batch_size=16, epochs=5, distributed=True)
        w = torch.cat([p.detach().float().flatten() for p in f.module.parameters()])
        q.put((rank, before, f.evaluate(x, y)[0], w.numpy()))
    finally:
        dist.destroy_process_group()


def test_forecaster_distributed_fit_two_ranks():
    """fit(distributed=True) over a 2-rank gloo group: every rank ends with the same weights
    and a lower loss."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    (_, b0, a0, w0), (_, b1, a1, w1) = res
    np.testing.assert_allclose(w0, w1, atol=1e-6)
    assert a0 < b0 and a1 < b1


def test_autots_fit_predict_save_load(tmp_path):
    from zoo.automl.config.recipe import SmokeRecipe
    from zoo.zouwu.autots.forecast import AutoTSTrainer, TSPipeline
    df = pd.DataFrame({"datetime": pd.date_range("2020-01-01", periods=120, freq="h"),
                       "value": np.sin(np.arange(120) / 6.0)})
    trainer = AutoTSTrainer(horizon=1, dt_col="datetime", target_col="value")
    ppl = trainer.fit(df[:100], df[100:], recipe=SmokeRecipe())
    assert len(ppl.predict(df[100:])) == 19
    f = str(tmp_path / "ts.ppl")
    ppl.save(f)
    new = TSPipeline.load(f)
    np.testing.assert_array_almost_equal(new.predict(df[100:])["value"].values,
                                         ppl.predict(df[100:])["value"].values, decimal=4)
    new.fit(df[:100], epochs=1)
    assert len(new.evaluate(df[100:], metrics=["mse"])) == 1
