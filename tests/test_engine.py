"""Training engine tests on CPU (the analogue of DistriEstimatorSpec /
TrainingSpec): convergence on toy problems, clipping,
iteration/epoch counters, triggers, checkpoint + failure retry with fault
injection, FeatureSet sharding / tiers, TensorBoard, and multi-process
data parallelism over gloo (world_size 2) for both gradient-sync modes."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from zoo.common import triggers as T
from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


def _mlp(seed=0):
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(seed)
    m = Sequential()
    m.add(Dense(8, activation="tanh", input_shape=(4,)))
    m.add(Dense(1))
    return m


def _toy(n=256, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, 4)).astype(np.float32)
    y = (x @ np.array([[1.0], [-2.0], [0.5], [3.0]], dtype=np.float32) + 0.3).astype(np.float32)
    return x, y


def test_mse_convergence_sgd():
    x, y = _toy()
    m = _mlp()
    from zoo.pipeline.api.keras.optimizers import SGD
    m.compile(optimizer=SGD(learningrate=0.05, momentum=0.9), loss="mse")
    before = m.evaluate(x, y)[0]
    m.fit(x, y, batch_size=32, nb_epoch=20)
    after = m.evaluate(x, y)[0]
    assert after < 0.05 * before, (before, after)


def test_iteration_and_epoch_counters():
    x, y = _toy(128)
    m = _mlp()
    m.compile(optimizer="sgd", loss="mse")
    m.fit(x, y, batch_size=32, nb_epoch=2)
    eng = m._engine
    assert eng.state["neval"] == 1 + 2 * (128 // 32)
    assert eng.state["epoch"] == 3
    m.fit(x, y, batch_size=32, nb_epoch=1)  # "train multi times" continues the counters
    assert eng.state["neval"] == 1 + 3 * 4 and m.get_finished_epoch() == 3


def test_gradient_clipping_constant_and_l2():
    x, y = _toy(64)
    for setup in ("const", "l2"):
        m = _mlp()
        m.compile(optimizer="sgd", loss="mse")
        if setup == "const":
            m.set_constant_gradient_clipping(-1e-3, 1e-3)
        else:
            m.set_gradient_clipping_by_l2_norm(1e-3)
        w0 = [p.detach().clone() for p in m.parameters()]
        eng = m._get_engine()
        eng.train_step(torch.from_numpy(x), torch.from_numpy(y))
        g = eng.flat.grad
        if setup == "const":
            assert g.abs().max().item() <= 1e-3 + 1e-9
        else:
            assert g.norm().item() <= 1e-3 * 1.01
        delta = max((p.detach() - q).abs().max().item() for p, q in zip(m.parameters(), w0))
        assert delta <= 0.01 * 1e-3 * 1.01 + 1e-9  # lr 0.01


def test_triggers():
    s = {"epoch": 3, "neval": 11, "Loss": 0.2, "score": 0.9, "epoch_end": True}
    assert T.MaxEpoch(2)(s) and not T.MaxEpoch(3)(s)
    assert T.MaxIteration(10)(s) and not T.MaxIteration(11)(s)
    assert T.SeveralIteration(5)(s)
    assert T.EveryEpoch()(s)
    assert T.MinLoss(0.3)(s) and not T.MinLoss(0.1)(s)
    assert T.MaxScore(0.8)(s)
    assert T.And(T.MaxEpoch(2), T.MinLoss(0.3))(s)
    assert T.Or(T.MaxEpoch(5), T.MinLoss(0.3))(s)


def test_checkpoint_and_failure_retry(tmp_path, monkeypatch):
    """Topology.scala:1180-1262: a failure mid-training reloads the latest
    checkpoint and continues (fault injected at iteration 6)."""
    from zoo.pipeline.engine import TrainingEngine
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.feature.common import FeatureSet
    x, y = _toy(128)
    m = _mlp()
    eng = TrainingEngine(m, MeanSquaredError(), SGD(learningrate=0.05))
    eng.set_checkpoint(str(tmp_path / "ckpt"), T.EveryEpoch(), overwrite=False)
    eng.fault_step = 6
    data = FeatureSet.from_ndarrays(x, y, 32)
    eng.fit(data, end_trigger=T.MaxEpoch(3))
    assert eng._fault_fired
    files = sorted(os.listdir(tmp_path / "ckpt"))
    assert any(f.startswith("model.") for f in files) and any(f.startswith("optimMethod-SGD.") for f in files)
    assert eng.state["epoch"] == 4


def test_failure_without_checkpoint_raises():
    from zoo.pipeline.engine import InjectedFault, TrainingEngine
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.feature.common import FeatureSet
    x, y = _toy(64)
    eng = TrainingEngine(_mlp(), MeanSquaredError(), SGD())
    eng.fault_step = 2
    with pytest.raises(InjectedFault):
        eng.fit(FeatureSet.from_ndarrays(x, y, 32), end_trigger=T.MaxEpoch(2))


def test_optim_method_save_load(tmp_path):
    from zoo.pipeline.api.keras.optimizers import Adam, OptimMethod
    o = Adam(lr=0.01)
    p = torch.randn(10)
    o.step(p, torch.randn(10))
    o.save(str(tmp_path / "adam"))
    o2 = OptimMethod.load(str(tmp_path / "adam"))
    assert isinstance(o2, Adam) and o2.state["neval"] == 2
    assert torch.allclose(o2._buffers[0], o._buffers[0])


def test_lr_schedules():
    from zoo.pipeline.api.keras import optimizers as O
    s = {"neval_prev": 10, "epoch": 3}
    assert O.Poly(0.5, 100).rate(1.0, s) == pytest.approx((1 - 0.1) ** 0.5)
    assert O.Step(5, 0.1).rate(1.0, s) == pytest.approx(0.01)
    assert O.MultiStep([5, 20], 0.1).rate(1.0, s) == pytest.approx(0.1)
    assert O.PolyEpochDecay(2, 10).rate(1.0, s) == pytest.approx(0.7 ** 2)
    seq = O.SequentialSchedule().add(O.Warmup(0.1), 5).add(O.Poly(1.0, 100), 100)
    assert seq.rate(0.0, {"neval_prev": 2, "epoch": 1}) == pytest.approx(0.2)
    sgd = O.SGD(learningrate=0.1, learningrate_decay=0.5)
    sgd.state["neval"] = 3
    assert sgd.current_lr() == pytest.approx(0.1 / (1 + 2 * 0.5))


def test_featureset_tiers_and_sharding(tmp_path):
    from zoo.feature.common import FeatureSet, MemoryType
    x = np.arange(100, dtype=np.float32).reshape(50, 2)
    y = np.arange(50, dtype=np.int64)
    for mt in (MemoryType.DRAM, MemoryType.DIRECT, MemoryType.DEVICE):
        fs = FeatureSet.from_ndarrays(x, y, 10, memory_type=mt)
        seen = []
        for bx, by in fs.data(train=True, epoch=1):
            assert bx.shape == (10, 2)
            assert torch.equal(bx[:, 0].long().cpu(), (by * 2).cpu())
            seen.extend(by.tolist())
        assert len(set(seen)) == 50
        ev = [b[1] for b in fs.data(train=False)]
        assert torch.equal(torch.cat(ev).cpu(), torch.arange(50))
    sl = FeatureSet.from_ndarrays(x, y, 10, memory_type=MemoryType.DISK_AND_DRAM(5))
    assert sl.num_of_slice() == 5 and sum(1 for _ in sl.data(train=True, epoch=0)) == 1


def test_tensorboard_roundtrip(tmp_path):
    from zoo.tensorboard import TrainSummary
    s = TrainSummary(str(tmp_path), "app")
    for i in range(5):
        s.add_scalar("Loss", 1.0 / (i + 1), i)
    s.add_histogram("w", np.random.randn(100), 1)
    vals = s.read_scalar("Loss")
    assert [v[0] for v in vals] == list(range(5))
    assert vals[2][1] == pytest.approx(1 / 3, rel=1e-6)
    s.close()


def test_keras_tensorboard_and_checkpoint(tmp_path):
    x, y = _toy(64)
    m = _mlp()
    m.compile(optimizer="sgd", loss="mse")
    m.set_tensorboard(str(tmp_path), "zoo")
    m.set_checkpoint(str(tmp_path / "ck"))
    os.environ["ZOO_LOG_EVERY"] = "1"
    m._engine = None
    m.fit(x, y, batch_size=16, nb_epoch=2)
    assert len(m.get_train_summary("Loss")) >= 1
    assert os.path.exists(tmp_path / "ck" / "model")


# ----------------------------------------------------------------------------
# multi-process data parallel over gloo (world_size 2)
# ----------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker_compressed(rank, world, port, out_q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "ZOO_GRAD_COMPRESSION": "bf16"})
    import zoo.common.nncontext as nc
    nc._CTX = None
    ctx = nc.init_nncontext(backend="gloo")
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(64)
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9), ctx=ctx,
                         bucket_mb=0.0001)
    assert eng.sync.compress == "bf16"
    for step in range(3):
        sl = slice(rank * 8 + step * 16, rank * 8 + step * 16 + 8)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    out_q.put((rank, eng.flat.master.detach().cpu().numpy().copy()))
    ctx.stop()


def test_data_parallel_bf16_gradient_compression():
    """16-bit gradient transfer (HK24): ranks stay identical and track the fp32 run closely."""
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_dp_worker_compressed, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: torch.from_numpy(v) for r, v in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    assert torch.equal(res[0], res[1])
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(64)
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9))
    for step in range(3):
        sl = slice(step * 16, step * 16 + 16)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    assert (res[0] - eng.flat.master).abs().max() < 2e-2 * eng.flat.master.abs().max()


def _dp_worker(rank, world, port, mode, out_q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import zoo.common.nncontext as nc
    nc._CTX = None
    ctx = nc.init_nncontext(backend="gloo", sharded_optimizer=(mode == "sharded"))
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(64)
    m = _mlp(seed=rank)  # different init per rank: broadcast must fix it
    eng = TrainingEngine(m, MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9), ctx=ctx,
                         sharded=(mode == "sharded"), bucket_mb=0.0001)
    for step in range(3):
        sl = slice(rank * 8 + step * 16, rank * 8 + step * 16 + 8)  # each rank: its half of a 16-batch
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    # numpy, not a shared-memory tensor: the fd-backed storage dies with this process
    out_q.put((rank, eng.flat.master.detach().cpu().numpy().copy()))
    ctx.stop()


@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
def test_data_parallel_gloo_matches_single_process(mode):
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_dp_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: torch.from_numpy(v) for r, v in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    assert torch.allclose(res[0], res[1], atol=1e-6), "ranks diverged"
    # single process, full 16-sample batches, rank-0 init
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(64)
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9))
    for step in range(3):
        sl = slice(step * 16, step * 16 + 16)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    assert torch.allclose(res[0], eng.flat.master, atol=1e-5)


def test_flat_safetensors_checkpoint_roundtrip(tmp_path):
    """Fast native snapshot: master + optimizer state restored exactly; training
    continues identically to an uninterrupted run."""
    from zoo.pipeline.engine import TrainingEngine
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import Adam
    x, y = _toy(64)
    xs, ys = torch.from_numpy(x), torch.from_numpy(y)
    a = TrainingEngine(_mlp(seed=3), MeanSquaredError(), Adam(lr=0.01))
    for _ in range(3):
        a.train_step(xs[:32], ys[:32])
    p = a.save_flat_checkpoint(str(tmp_path / "snap.safetensors"))
    b = TrainingEngine(_mlp(seed=9), MeanSquaredError(), Adam(lr=0.01))
    b.load_flat_checkpoint(p)
    assert torch.equal(a.flat.master, b.flat.master) and b.state["neval"] == a.state["neval"]
    la = a.train_step(xs[32:], ys[32:])
    lb = b.train_step(xs[32:], ys[32:])
    assert torch.allclose(a.flat.master, b.flat.master, atol=1e-7) and torch.allclose(la, lb)


def test_phase_timing_and_debug_sync_are_inert_on_cpu():
    from zoo.pipeline.engine import TrainingEngine
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    x, y = _toy(32)
    eng = TrainingEngine(_mlp(), MeanSquaredError(), SGD(learningrate=0.01))
    eng.debug_sync = True
    eng.train_step(torch.from_numpy(x), torch.from_numpy(y))
    assert eng.phase_times() == {}


# ----------------------------------------------------------------------------
# round-3 checkpoint interop: restore-by-name, OptimMethod records, neval ordering
# ----------------------------------------------------------------------------
def test_checkpoint_roundtrip_with_unserialisable_layers(tmp_path):
    """A model with a Lambda layer and a wrapped torch module (constructor arguments the
    ``.model`` file cannot represent) reloads into the live model by layer name."""
    from zoo.pipeline.api.autograd import Lambda
    from zoo.pipeline.api.keras.layers import Dense, KerasLayerWrapper
    from zoo.pipeline.api.keras.models import Sequential
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    torch.manual_seed(0)
    m = Sequential()
    m.add(Dense(8, activation="tanh", input_shape=(4,)))
    m.add(Lambda(lambda t: t * 2.0))
    m.add(KerasLayerWrapper(torch.nn.Linear(8, 3)))
    m.add(Dense(1))
    x, y = _toy(32)
    eng = TrainingEngine(m, MeanSquaredError(), SGD(learningrate=0.05, momentum=0.9))
    eng.set_checkpoint(str(tmp_path / "ck"), overwrite=False)
    for _ in range(3):
        eng.train_step(torch.from_numpy(x), torch.from_numpy(y))
    eng.save_checkpoint()
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    mom = [b.clone() for b in eng.optim._buffers]
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    eng.optim.clear_history()
    eng.load_checkpoint(eng.latest_checkpoint())
    for k, v in m.state_dict().items():
        assert torch.allclose(v.float(), ref[k].float()), k
    assert all(torch.allclose(a, b) for a, b in zip(eng.optim._buffers, mom))


def test_optim_method_record_is_bigdl_protobuf(tmp_path):
    from zoo.utils.bigdl_model import is_bigdl_model_file, load_optim_method, save_optim_method
    from zoo.utils import bigdl_proto as P
    d = {"class": "SGD", "state": {"neval": 7, "epoch": 2, "Loss": 0.25, "tag": "x"},
         "hyper": {"learningrate": 0.1, "momentum": 0.9, "nesterov": True},
         "buffers": [torch.randn(13), torch.arange(5, dtype=torch.int64) * (1 << 40)]}
    p = str(tmp_path / "optimMethod-SGD.7")
    save_optim_method(d, p)
    assert is_bigdl_model_file(p)
    root, _ = P.load_bigdl_spec(p)
    assert root.type == "com.intel.analytics.bigdl.optim.SGD"
    assert root.attr["learningRate"] == pytest.approx(0.1) and root.attr["state.neval"] == 7
    e = load_optim_method(p)
    assert e["class"] == "SGD" and e["state"] == d["state"] and e["hyper"] == d["hyper"]
    assert torch.equal(e["buffers"][0], d["buffers"][0])
    assert e["buffers"][1].dtype == torch.int64 and torch.equal(e["buffers"][1], d["buffers"][1])


def test_int64_buffers_roundtrip_exactly(tmp_path):
    from zoo.utils.bigdl_model import load_bigdl_model, save_bigdl_model
    net = torch.nn.BatchNorm1d(3)
    net.num_batches_tracked.fill_((1 << 40) + 3)
    p = str(tmp_path / "bn.model")
    save_bigdl_model(net, p)
    net2 = torch.nn.BatchNorm1d(3)
    load_bigdl_model(p, model=net2)
    assert int(net2.num_batches_tracked) == (1 << 40) + 3


def test_latest_checkpoint_by_iteration_not_mtime(tmp_path):
    import time
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(32)
    eng = TrainingEngine(_mlp(), MeanSquaredError(), SGD(learningrate=0.05))
    ck = tmp_path / "ck"
    eng.set_checkpoint(str(ck), overwrite=False)
    for _ in range(3):
        eng.train_step(torch.from_numpy(x), torch.from_numpy(y))
        eng.save_checkpoint()
    files = sorted(f for f in os.listdir(ck) if f.startswith("model."))
    assert len(files) == 3
    # a restored copy: the OLDEST snapshot gets the newest mtime
    now = time.time()
    for i, f in enumerate(sorted(files, key=lambda f: int(f.split(".")[1]))):
        os.utime(ck / f, (now - 100 * i, now - 100 * i))
    assert eng.latest_checkpoint().endswith("model.%d" % max(int(f.split(".")[1]) for f in files))
