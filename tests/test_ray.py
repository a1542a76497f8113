"""zoo.ray: task/actor runtime and the distributed trainer (Py/ray tests:
test/zoo/ray/test_ray_on_local.py, test/zoo/ray/mxnet/test_mxnet_gluon.py)."""
import numpy as np
import pytest
import torch

from zoo.ray import RayContext, get, put, remote, resource_to_bytes, wait


def _square(x):
    return x * x


class Counter:
    def __init__(self, start):
        self.v = start

    def add(self, d):
        self.v += d
        return self.v

    def fail(self):
        raise ValueError("boom")


@pytest.fixture(scope="module")
def ray_ctx():
    ctx = RayContext(sc=None, object_store_memory="100m", num_ray_nodes=1, ray_node_cpu_cores=2)
    ctx.init()
    yield ctx
    ctx.stop()


def test_resource_to_bytes():
    assert resource_to_bytes("50b") == 50
    assert resource_to_bytes("100k") == 100000
    assert resource_to_bytes("2g") == 2 * 10 ** 9
    with pytest.raises(ValueError):
        resource_to_bytes("1.5g")


def test_remote_functions_and_actors(ray_ctx):
    f = remote(_square)
    refs = [f.remote(i) for i in range(6)]
    assert get(refs) == [i * i for i in range(6)]
    ready, rest = wait(refs, num_returns=6)
    assert len(ready) == 6 and not rest
    assert get(put(7)) == 7
    C = remote(Counter)
    a = C.remote(10)
    assert get([a.add.remote(1), a.add.remote(2)]) == [11, 13]  # in-order actor execution
    with pytest.raises(ValueError):
        get(a.fail.remote())
    assert get(a.add.remote(0)) == 13  # the actor survives a failed call
    RayContext.kill(a)
    assert RayContext.get() is ray_ctx


def _data_creator(config, kv):
    rng = np.random.RandomState(kv.rank)
    xs = rng.randn(64, 4).astype(np.float32)
    ys = (xs.sum(1) > 0).astype(np.int64)
    b = config["batch_size"]
    train = [(torch.from_numpy(xs[i:i + b]), torch.from_numpy(ys[i:i + b])) for i in range(0, 64, b)]
    return train, train


def _model_creator(config):
    return torch.nn.Sequential(torch.nn.Linear(4, 16), torch.nn.ReLU(), torch.nn.Linear(16, 2))


def _loss_creator(config):
    return "sparse_categorical_crossentropy"


def test_distributed_trainer_two_workers(ray_ctx):
    from zoo.ray.mxnet import MXNetTrainer, create_trainer_config
    cfg = create_trainer_config(batch_size=16, optimizer="adam", optimizer_params={"learning_rate": 0.05},
                                log_interval=2, seed=3, extra_config={"backend": "gloo"})
    tr = MXNetTrainer(cfg, _data_creator, _model_creator, _loss_creator, lambda c: ["accuracy"], num_workers=2)
    try:
        s1 = tr.train(nb_epoch=1)
        s2 = tr.train(nb_epoch=4)
        assert len(s1) == 2 and all("loss" in s for s in s1)
        assert s2[0]["loss"] < s1[0]["loss"] + 0.2
        # synchronous DP: both workers report the same globally-reduced validation metric
        acc = [s for s in s2[0] if "ccuracy" in s]
        assert acc and abs(s2[0][acc[0]] - s2[1][acc[0]]) < 1e-6
        assert s2[0][acc[0]] > 0.7
        w = tr.get_weights()
        assert set(w) == {"0.weight", "0.bias", "2.weight", "2.bias"}
    finally:
        tr.shutdown()
