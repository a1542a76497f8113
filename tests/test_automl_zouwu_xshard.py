"""AutoML / Zouwu / XShards (test_time_sequence_predictor.py, test_forecast.py,
test_shard.py analogues). Reference fixture: pyzoo/test/zoo/resources/xshard/*.csv."""
import os

import numpy as np
import pandas as pd
import pytest

from zoo.common.nncontext import init_nncontext

XS = "/root/reference/pyzoo/test/zoo/resources/xshard"


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _ts(n=300):
    dt = pd.date_range("2020-01-01", periods=n, freq="h")
    v = np.sin(np.arange(n) / 6.0) + 0.05 * np.random.default_rng(0).standard_normal(n)
    return pd.DataFrame({"datetime": dt, "value": v})


def test_metrics():
    from zoo.automl.common.metrics import Evaluator
    y = np.array([1.0, 2.0, 4.0])
    p = np.array([1.0, 2.5, 3.0])
    assert Evaluator.evaluate("mse", y, p, "uniform_average") == pytest.approx((0.25 + 1) / 3)
    assert Evaluator.evaluate("mae", y, p, "uniform_average") == pytest.approx(0.5)
    assert Evaluator.evaluate("r2", y, y, "uniform_average") == pytest.approx(1.0)
    assert Evaluator.evaluate("smape", y, y, "uniform_average") == pytest.approx(0.0)


def test_feature_transformer_rolling():
    from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
    df = _ts(50)
    ft = TimeSequenceFeatureTransformer(future_seq_len=2)
    x, y = ft.fit_transform(df, past_seq_len=4, selected_features=["HOUR(datetime)", "IS_WEEKEND(datetime)"])
    assert x.shape == (45, 4, 3) and y.shape == (45, 2)
    # target column is first; y is the scaled target of the next 2 steps
    assert np.allclose(x[1, -1, 0], y[0, 0])
    truth, back = ft.post_processing(df, y, True)
    assert np.allclose(back[:, 0], df["value"].values[4:49], atol=1e-6)
    assert np.allclose(truth, back, atol=1e-6)


def test_search_expand_grid_random():
    from zoo.automl.search import GridSearch, RandomSample, expand
    cfgs = expand({"a": GridSearch([1, 2]), "b": RandomSample(lambda s: s["a"] * 10), "c": 5}, num_samples=2)
    assert len(cfgs) == 4 and {c["b"] for c in cfgs} == {10, 20} and all(c["c"] == 5 for c in cfgs)


def test_time_sequence_predictor_fit_predict_save(tmp_path):
    from zoo.automl.config.recipe import LSTMGridRandomRecipe
    from zoo.automl.pipeline import load_ts_pipeline
    from zoo.automl.regression import TimeSequencePredictor
    df = _ts()
    train, val = df[:240], df[240:]
    tsp = TimeSequencePredictor(future_seq_len=1)
    recipe = LSTMGridRandomRecipe(num_rand_samples=1, epochs=3, training_iteration=2, look_back=6,
                                  lstm_1_units=[16], lstm_2_units=[8, 16], batch_size=[32])
    ppl = tsp.fit(train, val, metric="mse", recipe=recipe)
    assert len(tsp.trials) == 2
    mse = ppl.evaluate(val, ["mse"], "uniform_average")[0]
    assert mse < np.var(val["value"].values)
    pred = ppl.predict(val)
    assert list(pred.columns) == ["datetime", "value"] and len(pred) == len(val) - 6 + 1
    p = ppl.save(str(tmp_path / "ppl"))
    ppl2 = load_ts_pipeline(p)
    assert np.allclose(ppl2.predict(val)["value"].values, pred["value"].values, atol=1e-5)
    mean, unc = ppl.predict_with_uncertainty(val, n_iter=5)
    assert unc.shape[0] == len(mean)


def test_mtnet_and_seq2seq_models_forward():
    import torch
    from zoo.automl.model import LSTMSeq2SeqNet, MTNetNet
    x = torch.randn(4, 9, 3)
    assert MTNetNet(3, 2, time_step=3, long_num=2, ar_window=2)(x).shape == (4, 2)
    net = LSTMSeq2SeqNet(3, 1, latent_dim=8, past_seq_len=9)
    assert net.decode(x, 3).shape == (4, 3, 1)
    assert net(torch.cat([x, torch.zeros(4, 3, 3)], 1)).shape == (4, 3, 1)     # teacher-forced graph


def test_zouwu_forecasters_and_autots(tmp_path):
    from zoo.automl.config.recipe import SmokeRecipe
    from zoo.zouwu.autots import AutoTSTrainer, TSPipeline
    from zoo.zouwu.model import LSTMForecaster, MTNetForecaster
    rng = np.random.default_rng(1)
    x = rng.standard_normal((64, 6, 2)).astype(np.float32)
    y = x[:, -1, :1] * 0.5
    f = LSTMForecaster(horizon=1, feature_dim=2, lr=0.01)
    before = f.evaluate(x, y)[0]
    f.fit(x, y, batch_size=16, epochs=20)
    assert f.evaluate(x, y)[0] < before
    m = MTNetForecaster(horizon=1, feature_dim=2, lb_long_steps=2, lb_long_stepsize=2, ar_window=2, cnn_height=2)
    assert m.predict(m.preprocess_input(x)).shape == (64, 1)
    df = _ts(120)
    ppl = AutoTSTrainer(horizon=1).fit(df[:100], df[100:], recipe=SmokeRecipe())
    assert isinstance(ppl, TSPipeline) and len(ppl.predict(df[100:])) == 19
    ppl.save(str(tmp_path / "p"))
    assert len(TSPipeline.load(str(tmp_path / "p")).predict(df[100:])) == 19


def test_xshards_read_apply_repartition(tmp_path):
    from zoo import xshard
    if os.path.isdir(XS):
        shards = xshard.read_csv(XS)
        assert shards.num_partitions() >= 1 and len(shards.concat()) > 0
    for i in range(3):
        pd.DataFrame({"a": np.arange(i * 10, i * 10 + 10), "b": 1.0}).to_csv(tmp_path / ("p%d.csv" % i), index=False)
    s = xshard.read_csv(str(tmp_path))
    assert s.num_partitions() == 3
    s2 = s.apply(lambda df, k: df.assign(c=df["a"] * k), 2)
    assert s2.concat()["c"].sum() == 2 * np.arange(30).sum()
    r = s2.repartition(2)
    assert r.num_partitions() == 2 and len(r.concat()) == 30


def test_bayes_opt_beats_random_on_a_smooth_objective():
    """BayesOptSearch (GP + UCB) concentrates its samples near the optimum of a smooth
    2-D objective: its best after 20 evaluations beats the best of 20 uniform samples
    (averaged over seeds), and the engine's Bayes path converts bayes spaces."""
    import numpy as np
    from zoo.automl.search import BayesOptSearch, SearchEngine

    def f(p):
        return -((p["a"] - 0.3) ** 2 + (p["b"] - 0.7) ** 2)
    wins = 0
    for seed in range(4):
        opt = BayesOptSearch({"a": (0, 1), "b": (0, 1)}, seed=seed)
        for _ in range(20):
            pt = opt.suggest(1)[0]
            opt.observe(pt, f(pt))
        rng = np.random.default_rng(seed)
        rand_best = max(f({"a": rng.random(), "b": rng.random()}) for _ in range(20))
        wins += max(opt.y) > rand_best
    assert wins >= 3
    eng = SearchEngine()
    best_cfg, best = eng.run(lambda c: {"mse": (c["lstm_1_units"] - 64) ** 2 + c["batch_size"] * 0.0},
                             {"lstm_1_units_float": (8, 128), "batch_size_log": (5, 10)}, num_samples=8,
                             search_alg="BayesOpt", fixed_params={"epochs": 1})
    assert set(best_cfg) == {"lstm_1_units", "batch_size", "epochs"} and len(eng.trials) == 8
    assert 32 <= best_cfg["batch_size"] <= 1024 and isinstance(best_cfg["lstm_1_units"], int)


def test_time_sequence_predictor_with_bayes_recipe():
    import numpy as np
    import pandas as pd
    from zoo.automl.config.recipe import BayesRecipe
    from zoo.automl.regression.time_sequence_predictor import TimeSequencePredictor
    n = 80
    df = pd.DataFrame({"datetime": pd.date_range("2020-01-01", periods=n, freq="h"),
                       "value": np.sin(np.arange(n) / 5.0).astype(np.float32)})
    tsp = TimeSequencePredictor(future_seq_len=1)
    ppl = tsp.fit(df, recipe=BayesRecipe(num_samples=3, look_back=(2, 4), epochs=1, training_iteration=1))
    assert len(tsp.trials) == 3
    from zoo.automl.common.util import convert_bayes_configs
    cfgs = [convert_bayes_configs(t.config) for t in tsp.trials]          # raw GP points + fixed params
    assert all(2 <= c["past_seq_len"] <= 4 and c["model"] == "LSTM" for c in cfgs)
    assert all(t.last_result["training_iteration"] == 1 for t in tsp.trials)     # stop criterion
    assert ppl.predict(df).shape[0] > 0


def test_automl_base_models_fit_eval_save_restore(tmp_path):
    """BaseModel contract (Py/automl/model/abstract.py): fit_eval returns the validation
    metric, save/restore round-trips, TimeSequenceModel picks the model from the config."""
    from zoo.automl.model import LSTMSeq2Seq, MTNetKeras, TimeSequenceModel, VanillaLSTM
    rng = np.random.default_rng(3)
    x = rng.standard_normal((96, 6, 2)).astype(np.float32)
    y = (x[:, -1, :1] * 0.7 + 0.1).astype(np.float32)
    m = VanillaLSTM(check_optional_config=False, future_seq_len=1)
    first = m.fit_eval(x, y, validation_data=(x, y), lstm_1_units=8, lstm_2_units=4, lr=0.01, epochs=1)
    later = m.fit_eval(x, y, validation_data=(x, y), epochs=15)
    assert later < first
    m.save(str(tmp_path / "m.pt"), str(tmp_path / "m.json"))
    import json
    cfg = json.load(open(tmp_path / "m.json"))
    m2 = VanillaLSTM().restore(str(tmp_path / "m.pt"), **cfg)
    assert np.allclose(m2.predict(x), m.predict(x), atol=1e-5)
    mean, std = m.predict_with_uncertainty(x[:8], n_iter=4)
    assert mean.shape == (8, 1) and std.shape == (8, 1)
    with pytest.raises(ValueError, match="look-back"):     # defaults long_num 7, time_step 1 need 8 steps
        MTNetKeras().fit_eval(x, y, epochs=1)
    mt = MTNetKeras(future_seq_len=1)
    assert mt.fit_eval(x, y, long_num=2, time_step=2, epochs=1) >= 0
    tsm = TimeSequenceModel(future_seq_len=2)
    y2 = np.concatenate([y, y], 1)
    tsm.fit_eval(x, y2, latent_dim=8, epochs=1)
    assert tsm.selected_model == "Seq2seq" and tsm.predict(x).shape == (96, 2)
    assert isinstance(tsm.model, LSTMSeq2Seq)


def test_search_engine_abstract_contract():
    from zoo.automl.search import GridSearch, RandomSample, SearchEngine
    from zoo.automl.search.RayTuneSearchEngine import RayTuneSearchEngine
    from zoo.automl.search.abstract import SearchEngine as Abstract
    assert issubclass(SearchEngine, Abstract) and issubclass(RayTuneSearchEngine, Abstract)
    eng = SearchEngine()
    space = {"a": GridSearch([1, 2, 3]), "b": RandomSample(lambda spec: spec["a"] * 10)}
    best_cfg, best = eng.run(lambda c: {"mse": abs(c["a"] - 2) + 0.0 * c["b"]}, space)
    assert best_cfg == {"a": 2, "b": 20}
    assert [c["a"] for c in eng.get_best_trials(2)] in ([2, 1], [2, 3])
