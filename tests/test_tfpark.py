"""TFPark API on the engine (test_tf_optimizer.py / test_tfpark_model.py /
test_gan_estimator.py / GanOptimMethodSpec analogues)."""
import numpy as np
import pandas as pd
import pytest
import torch

from zoo.common import triggers as T
from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _data(n=128):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((n, 5)).astype(np.float32)
    return x, (x[:, :1] * 2 - x[:, 1:2]).astype(np.float32)


def _net():
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(0)
    m = Sequential()
    m.add(Dense(16, activation="relu", input_shape=(5,)))
    m.add(Dense(1))
    return m


def test_keras_model_fit_evaluate_predict_batches(tmp_path):
    from zoo.tfpark import KerasModel, TFDataset
    x, y = _data()
    from zoo.pipeline.api.keras.optimizers import Adam
    km = KerasModel(_net(), optimizer=Adam(lr=0.01), loss="mse")
    before = km.evaluate(x, y)[0]
    km.fit(TFDataset.from_ndarrays((x, y), batch_size=16, val_tensors=(x, y)), epochs=15)
    assert km.evaluate(x, y)[0] < 0.3 * before
    assert km.predict(x).shape == (128, 1)
    l0 = km.train_on_batch(x[:16], y[:16])
    assert np.isfinite(l0)
    km.save_weights(str(tmp_path / "w"))
    w = km.get_weights()
    km.set_weights([np.zeros_like(a) for a in w])
    km.load_weights(str(tmp_path / "w"))
    assert all(np.allclose(a, b) for a, b in zip(km.get_weights(), w))


def test_tfoptimizer_from_keras_and_dataframe():
    from zoo.tfpark import KerasModel, TFDataset, TFOptimizer
    x, y = _data(64)
    df = pd.DataFrame({"f": list(x), "label": y[:, 0]})
    ds = TFDataset.from_dataframe(df, ["f"], ["label"], batch_size=16)
    m = _net()
    m.compile("sgd", "mse")
    before = m.evaluate(x, y[:, 0])[0]
    opt = TFOptimizer.from_keras(m, ds, optim_method="adam")
    opt.set_gradient_clipping_by_l2_norm(10.0)
    opt.optimize(T.MaxEpoch(10))
    assert m.evaluate(x, y[:, 0])[0] < before
    with pytest.raises(TypeError, match="TFNet"):
        TFOptimizer.from_loss(None, None)


def test_tfestimator_model_fn():
    from zoo.tfpark import TFEstimator, TFEstimatorSpec
    x, y = _data(64)
    lin = torch.nn.Linear(5, 1)

    def model_fn(features, labels, mode, params):
        pred = lin(features)
        loss = None if labels is None else torch.nn.functional.mse_loss(pred, labels)
        return TFEstimatorSpec(mode, pred, loss)

    def input_fn():
        for i in range(0, 64, 16):
            yield torch.from_numpy(x[i:i + 16]), torch.from_numpy(y[i:i + 16])
    from zoo.pipeline.api.keras.optimizers import Adam
    est = TFEstimator.from_model_fn(model_fn, [lin], optimizer=Adam(lr=0.05))
    before = est.evaluate(input_fn)["loss"]
    est.train(input_fn, steps=200)
    assert est.evaluate(input_fn)["loss"] < 0.2 * before
    assert est.predict(input_fn).shape == (64, 1)


def test_gan_optim_method_schedule():
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.tfpark import GanOptimMethod
    om = GanOptimMethod(SGD(learningrate=1.0), SGD(learningrate=1.0), d_steps=2, g_steps=1, g_param_size=3)
    master = torch.zeros(8)
    for k in range(3):
        om.step(master, torch.ones(8))
    # two D steps moved the tail, one G step the head
    assert torch.allclose(master[:3], -torch.ones(3)) and torch.allclose(master[3:], -2 * torch.ones(5))


def test_gan_estimator_learns_mean():
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.tfpark import GANEstimator
    torch.manual_seed(0)
    G = torch.nn.Sequential(torch.nn.Linear(2, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1))
    D = torch.nn.Sequential(torch.nn.Linear(1, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1))
    bce = torch.nn.functional.binary_cross_entropy_with_logits

    def g_loss(fake_logits):
        return bce(fake_logits, torch.ones_like(fake_logits))

    def d_loss(real_logits, fake_logits):
        return bce(real_logits, torch.ones_like(real_logits)) + bce(fake_logits, torch.zeros_like(fake_logits))
    est = GANEstimator(G, D, g_loss, d_loss, Adam(lr=5e-3), Adam(lr=5e-3), noise_dim=2)
    real = torch.randn(4096, 1) * 0.5 + 3.0
    data = [real[i:i + 64] for i in range(0, 4096, 64)]
    est.train(data, 1200)
    gen = est.generate(2000)
    assert abs(float(gen.mean()) - 3.0) < 0.6, float(gen.mean())


def test_tfdataset_string_bytes_and_rdd_sources():
    """TFDataset.from_string_rdd / from_bytes_rdd (batches of byte strings, the reference's
    single tf.string feature) and from_rdd over sample collections (list or collect())."""
    import numpy as np
    from zoo.tfpark import TFDataset
    strs = ["s%d,%d" % (i, i % 3) for i in range(10)]
    ds = TFDataset.from_string_rdd(strs, batch_per_thread=4)
    batches = [b[0] for b in ds.get_prediction_data().data(train=False)]
    assert [len(b) for b in batches] == [4, 4, 2] and batches[0][0] == b"s0,0"
    tr = TFDataset.from_bytes_rdd([s.encode() for s in strs], batch_size=4, hard_code_batch_size=True,
                                  validation_bytes_rdd=[b"v"])
    got = [x for b in tr.get_training_data().data(train=True, epoch=1) for x in b[0]]
    assert len(got) == 8 and set(got) <= {s.encode() for s in strs}   # shuffled, last partial dropped
    assert [b[0] for b in tr.get_validation_data().data(train=False)] == [[b"v"]]

    class FakeRDD:
        def __init__(self, items):
            self.items = items

        def collect(self):
            return list(self.items)
    samples = [(np.full(3, i, np.float32), np.int64(i % 2)) for i in range(8)]
    rd = TFDataset.from_rdd(FakeRDD(samples), batch_per_thread=8)
    x, y = next(iter(rd.get_prediction_data().data(train=False)))
    assert tuple(np.asarray(x).shape) == (8, 3) and list(np.asarray(y)) == [i % 2 for i in range(8)]


def _linreg_graph(tmp_path, with_train_op=None):
    """x [N, 3] -> pred = x @ w + b; loss = mean((pred - y)^2); variables with Assign initialisers."""
    import numpy as np
    from zoo.util.tf import graph_def, node_def
    F32 = ("type", 1)
    nodes = [
        node_def("x", "Placeholder", dtype=F32, shape=("shape", [-1, 3])),
        node_def("y", "Placeholder", dtype=F32, shape=("shape", [-1, 1])),
        node_def("w", "VariableV2", dtype=F32, shape=("shape", [3, 1])),
        node_def("w/init", "Const", dtype=F32, value=np.zeros((3, 1), np.float32)),
        node_def("w/Assign", "Assign", ["w", "w/init"], T=F32),
        node_def("b", "VariableV2", dtype=F32, shape=("shape", [1])),
        node_def("b/init", "Const", dtype=F32, value=np.zeros((1,), np.float32)),
        node_def("b/Assign", "Assign", ["b", "b/init"], T=F32),
        node_def("mm", "MatMul", ["x", "w"], T=F32, transpose_a=False, transpose_b=False),
        node_def("pred", "Add", ["mm", "b"], T=F32),
        node_def("diff", "Sub", ["pred", "y"], T=F32),
        node_def("sq", "Square", ["diff"], T=F32),
        node_def("axes", "Const", dtype=("type", 3), value=np.array([0, 1], np.int32)),
        node_def("loss", "Mean", ["sq", "axes"], T=F32, Tidx=("type", 3), keep_dims=False),
    ]
    if with_train_op:
        nodes += [node_def("lr", "Const", dtype=F32, value=np.array(0.1, np.float32)),
                  node_def("grad_w", "Identity", ["w"], T=F32),
                  node_def("grad_b", "Identity", ["b"], T=F32),
                  node_def("upd_w", "ApplyGradientDescent", ["w", "lr", "grad_w"], T=F32),
                  node_def("upd_b", "ApplyGradientDescent", ["b", "lr", "grad_b"], T=F32),
                  node_def("train", "NoOp", ["^upd_w", "^upd_b"])]
    p = tmp_path / "graph.pb"
    p.write_bytes(graph_def(nodes))
    return str(p)


def test_tfoptimizer_from_loss_trains_graph_variables(tmp_path):
    """In-graph loss (TFOptimizer.from_loss): the graph's variables are trained through the
    TF-graph executor + autograd + the native fused optimizer."""
    import numpy as np
    from zoo.common import triggers as T
    from zoo.tfpark.tf_optimizer import TFOptimizer
    from zoo.tfpark.tfnet import TFNet
    r = np.random.RandomState(0)
    x = r.randn(256, 3).astype(np.float32)
    y = (x @ np.array([[1.5], [-2.0], [0.5]], np.float32) + 0.3).astype(np.float32)
    net = TFNet(_linreg_graph(tmp_path), ["x:0", "y:0"], ["loss:0"], trainable=True)
    batches = [(x[i:i + 32], y[i:i + 32]) for i in range(0, 256, 32)]
    from zoo.pipeline.api.keras.optimizers import Adam
    opt = TFOptimizer.from_loss(net, Adam(lr=0.05), dataset=batches)
    opt.optimize(end_trigger=T.MaxEpoch(40))
    assert opt.losses[-1] < 0.05 * opt.losses[0]
    w = dict(net.named_parameters())
    vals = sorted(float(v) for p in w.values() for v in p.detach().cpu().reshape(-1))
    assert abs(vals[0] + 2.0) < 0.3 and abs(vals[-1] - 1.5) < 0.3


def test_tfoptimizer_from_train_op_uses_graph_optimizer(tmp_path):
    import numpy as np
    from zoo.common import triggers as T
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.tfpark.tf_optimizer import TFOptimizer
    from zoo.tfpark.tfnet import TFNet
    r = np.random.RandomState(1)
    x = r.randn(128, 3).astype(np.float32)
    y = (x @ np.array([[1.0], [1.0], [1.0]], np.float32)).astype(np.float32)
    net = TFNet(_linreg_graph(tmp_path, with_train_op=True), ["x:0", "y:0"], ["loss:0"], trainable=True)
    opt = TFOptimizer.from_train_op("train", net, dataset=[(x[i:i + 32], y[i:i + 32]) for i in range(0, 128, 32)])
    assert isinstance(opt.optim, SGD) and abs(opt.optim.current_lr() - 0.1) < 1e-7
    opt.optimize(end_trigger=T.MaxEpoch(20))
    assert opt.losses[-1] < 0.01 * opt.losses[0]
