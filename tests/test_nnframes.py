"""NNFrames on pandas DataFrames (NNEstimatorSpec / NNClassifierSpec /
NNImageReaderSpec analogues)."""
import numpy as np
import pandas as pd
import pytest
import torch

from zoo.common import triggers as T
from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _df(n=200, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, 4)).astype(np.float32)
    lab = np.where(x[:, 0] - x[:, 2] > 0, 2.0, 1.0)  # 1-based labels like the reference examples
    return pd.DataFrame({"features": list(x), "label": lab})


def _net(out=2, act="log_softmax"):
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(0)
    m = Sequential()
    m.add(Dense(12, activation="tanh", input_shape=(4,)))
    m.add(Dense(out, activation=act))
    return m


def test_nnclassifier_fit_transform_save_load(tmp_path):
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.nnframes import NNClassifier, NNClassifierModel
    df = _df()
    clf = NNClassifier(_net(), ClassNLLCriterion(), [4]).setBatchSize(32).setMaxEpoch(15) \
        .setOptimMethod(Adam(lr=0.05)).setValidation(T.EveryEpoch(), df, ["accuracy"], 64)
    model = clf.fit(df)
    out = model.transform(df)
    acc = (out["prediction"].values == df["label"].values).mean()
    assert acc > 0.9 and set(np.unique(out["prediction"])) <= {1.0, 2.0}
    model.save(str(tmp_path / "m"))
    m2 = NNClassifierModel.load(str(tmp_path / "m"))
    out2 = m2.transform(df)
    assert (out2["prediction"].values == out["prediction"].values).all()


def test_nnestimator_regression_and_cache_levels():
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.nnframes import NNEstimator
    rng = np.random.default_rng(1)
    x = rng.standard_normal((128, 4)).astype(np.float32)
    y = (x @ np.array([1.0, -1.0, 0.5, 2.0], np.float32)).reshape(-1, 1)
    df = pd.DataFrame({"f": list(x), "y": list(y)})
    for level in ("DRAM", "DEVICE"):
        est = NNEstimator(_net(1, None), MeanSquaredError(), [4], [1]).setFeaturesCol("f").setLabelCol("y") \
            .setLearningRate(0.1).setMaxEpoch(30).setBatchSize(16).setDataCacheLevel(level)
        model = est.fit(df)
        pred = np.array(model.setPredictionCol("p").transform(df)["p"].tolist())
        assert pred.shape == (128, 1)
        assert np.mean((pred - y) ** 2) < 0.3 * np.var(y)


def test_binary_threshold_prediction():
    from zoo.pipeline.nnframes import NNClassifierModel
    m = NNClassifierModel(_net(1, "sigmoid"), [4]).setThreshold(0.5)
    out = m.transform(_df(10))
    assert set(out["prediction"]) <= {0.0, 1.0}


def test_nn_image_reader(tmp_path):
    from PIL import Image
    from zoo.pipeline.nnframes import NNImageReader
    from zoo.pipeline.nnframes.nn_image_reader import row_to_array
    rgb = np.zeros((5, 7, 3), np.uint8)
    rgb[..., 0] = 200  # red
    Image.fromarray(rgb).save(tmp_path / "a.png")
    Image.fromarray(rgb[:, :, 0]).save(tmp_path / "b.png")
    df = NNImageReader.readImages(str(tmp_path))
    assert len(df) == 2
    r = df["image"][0]
    assert (r["height"], r["width"], r["nChannels"], r["mode"]) == (5, 7, 3, 16)
    assert row_to_array(r)[0, 0].tolist() == [0, 0, 200]  # BGR order
    assert df["image"][1]["nChannels"] == 1
    df2 = NNImageReader.readImages(str(tmp_path / "*.png"), resizeH=4, resizeW=4)
    assert df2["image"][0]["height"] == 4
