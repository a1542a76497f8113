"""Estimator / LocalEstimator / Predictor (EstimatorSpec, LocalEstimatorSpec,
PredictorSpec analogues)."""
import numpy as np
import pytest
import torch

from zoo.common import triggers as T
from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _data(n=256, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, 6)).astype(np.float32)
    y = (x[:, 0] + 0.5 * x[:, 1] > 0).astype(np.int64)
    return x, y


def _model(seed=0):
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(seed)
    m = Sequential()
    m.add(Dense(16, activation="relu", input_shape=(6,), name="hidden"))
    m.add(Dense(2, activation="log_softmax", name="head"))
    return m


def test_estimator_train_evaluate_checkpoint(tmp_path):
    from zoo.feature.common import FeatureSet
    from zoo.pipeline.api.keras.metrics import Accuracy
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.estimator import Estimator
    x, y = _data()
    est = Estimator(_model(), Adam(lr=0.02), model_dir=str(tmp_path / "ck"))
    fs = FeatureSet.from_ndarrays(x, y, 32)
    est.train(fs, ClassNLLCriterion(), end_trigger=T.MaxEpoch(6), checkpoint_trigger=T.EveryEpoch(),
              validation_set=FeatureSet.from_ndarrays(x, y, 64, shuffle=False), validation_method=[Accuracy()])
    res = est.evaluate(FeatureSet.from_ndarrays(x, y, 64, shuffle=False), [Accuracy()])
    assert res["Accuracy"] > 0.9
    import os
    assert any(f.startswith("model") for f in os.listdir(tmp_path / "ck"))


def test_estimator_clipping_and_per_submodule_optim():
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.estimator import Estimator
    x, y = _data(64)
    m = _model()
    w_hidden = m.get_layer("hidden").weight.detach().clone()
    w_head = m.get_layer("head").weight.detach().clone()
    # hidden layer frozen (lr 0), head trained
    est = Estimator(m, {"hidden": SGD(learningrate=0.0), "head": SGD(learningrate=0.5)})
    est.set_l2_norm_gradient_clipping(10.0)
    est.train((x, y), ClassNLLCriterion(), end_trigger=T.MaxIteration(3), batch_size=32)
    assert torch.equal(m.get_layer("hidden").weight.detach().cpu(), w_hidden.cpu())
    assert not torch.equal(m.get_layer("head").weight.detach().cpu(), w_head.cpu())


def test_local_estimator_slices_match_full_batch():
    """thread_num slices of equal size: averaged slice gradients == full-batch gradient."""
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.estimator import LocalEstimator
    x, y = _data(48)
    xs, ys = torch.from_numpy(x), torch.from_numpy(y)
    res = []
    for tn in (1, 4):
        le = LocalEstimator(_model(), ClassNLLCriterion(), SGD(learningrate=0.1), thread_num=tn, device="cpu")
        for _ in range(3):
            le.optimize(xs, ys)
        res.append(le.flat.master.clone())
    assert torch.allclose(res[0], res[1], atol=1e-6)
    le = LocalEstimator(_model(), ClassNLLCriterion(), SGD(learningrate=0.5), validations=["accuracy"],
                        thread_num=3, device="cpu")
    le.fit([(x[i:i + 16], y[i:i + 16]) for i in range(0, 48, 16)] * 2, epochs=10)
    acc = dict(le.validate([(x, y)]))
    assert list(acc.values())[0] > 0.85


def test_predictor_matches_forward():
    from zoo.pipeline.estimator import Predictor
    x, _ = _data(70)
    m = _model()
    p = Predictor(m, batch_per_thread=16, device="cpu")
    out = p.predict(x)
    with torch.no_grad():
        ref = m(torch.from_numpy(x)).numpy()
    assert out.shape == (70, 2) and np.allclose(out, ref, atol=1e-6)
    assert (p.predict_classes(x) == ref.argmax(-1)).all()
