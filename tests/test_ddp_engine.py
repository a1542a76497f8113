"""Data-parallel engine correctness (round 2): shared-parameter bucket launch,
ZeRO-1 with per-part optimizers and 16-bit wire format, per-rank sharded
checkpoints, cross-rank failure agreement, tensor parallelism through the engine.
All multi-rank cases run over gloo with world_size 2 (CPU)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch
import torch.nn as nn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mlp(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(6, 16), nn.Tanh(), nn.Linear(16, 8), nn.Tanh(), nn.Linear(8, 1))


def _toy(n=64, seed=1):
    r = np.random.RandomState(seed)
    x = r.randn(n, 6).astype(np.float32)
    y = (np.sin(x[:, :1]) + 0.1 * x[:, 1:2]).astype(np.float32)
    return x, y


def _init(rank, world, port, **env):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    for k, v in env.items():
        os.environ[k] = str(v)
    import zoo.common.nncontext as nc
    nc._CTX = None
    return nc.init_nncontext(backend="gloo")


def _run(target, *args, world=2, timeout=240):
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=timeout) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


# ---------------------------------------------------------------------------
# shared parameters: a bucket launches only after the LAST contribution
# ---------------------------------------------------------------------------
def test_shared_parameter_bucket_waits_for_every_contribution():
    import torch.distributed as dist
    from zoo.parallel.ddp import GradSync
    from zoo.parallel.flat import FlatParams
    dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
    try:
        lin, other = nn.Linear(4, 4), nn.Linear(4, 2)
        flat = FlatParams(list(lin.parameters()) + list(other.parameters()))
        sync = GradSync(flat, bucket_mb=1.0, force_comm=True)
        sync.overlap = True  # the CPU path is synchronous; drive the launch logic directly
        launches = []
        sync._issue = lambda b: launches.append(b.idx)
        assert len(sync.buckets) == 1

        def backward_pass():
            # lin.weight is used twice (a shared layer): two contributions
            for p in (other.weight, other.bias, lin.weight, lin.bias, lin.weight):
                sync._ready(p)
        backward_pass()                     # calibration step: nothing launches early
        assert launches == []
        sync.finish()
        assert launches == [0]
        sync.reset()
        launches.clear()
        for p in (other.weight, other.bias, lin.weight, lin.bias):
            sync._ready(p)
        assert launches == [], "bucket launched before the shared weight's second contribution"
        sync._ready(lin.weight)
        assert launches == [0]
        sync.finish()                       # nothing left to launch
        assert launches == [0]
        sync.reset()
        # a step with MORE contributions than calibrated after the launch must fail loudly
        launches.clear()
        for p in (other.weight, other.bias, lin.weight, lin.bias, lin.weight):
            sync._ready(p)
        with pytest.raises(RuntimeError, match="calibration"):
            sync._ready(lin.weight)
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# ZeRO-1: per-submodule optimizers and the bf16 all-to-all wire format
# ---------------------------------------------------------------------------
def _zero1_worker(rank, world, port, q, compress, multi):
    ctx = _init(rank, world, port, ZOO_GRAD_COMPRESSION=compress)
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD, Adam
    from zoo.pipeline.engine import TrainingEngine
    from zoo.pipeline.estimator.estimator import MultiOptimMethod
    x, y = _toy(64)
    m = _mlp(seed=0)
    eng = TrainingEngine(m, MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9), ctx=ctx, sharded=True,
                         bucket_mb=0.0003)
    if multi:
        from zoo.pipeline.estimator.estimator import _resolve_optim
        eng.optim = _resolve_optim(m, {"0": Adam(lr=0.01), "2": SGD(learningrate=0.1), "4": SGD(learningrate=0.05)},
                                   eng.flat)
        assert isinstance(eng.optim, MultiOptimMethod)
    for step in range(4):
        sl = slice(rank * 8 + step * 16, rank * 8 + step * 16 + 8)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    eng.sync.sync_master()
    q.put((rank, eng.flat.master.detach().numpy().copy()))
    ctx.stop()


@pytest.mark.parametrize("compress,multi", [("", True), ("bf16", False), ("bf16", True)])
def test_zero1_matches_single_process(compress, multi):
    res = _run(_zero1_worker, compress, multi)
    r0, r1 = torch.from_numpy(res[0]), torch.from_numpy(res[1])
    assert torch.allclose(r0, r1, atol=1e-6), "ranks diverged"
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD, Adam
    from zoo.pipeline.engine import TrainingEngine
    from zoo.pipeline.estimator.estimator import _resolve_optim
    x, y = _toy(64)
    m = _mlp(seed=0)
    eng = TrainingEngine(m, MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9))
    if multi:
        eng.optim = _resolve_optim(m, {"0": Adam(lr=0.01), "2": SGD(learningrate=0.1), "4": SGD(learningrate=0.05)},
                                   eng.flat)
    for step in range(4):
        sl = slice(step * 16, step * 16 + 16)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    tol = 2e-2 * eng.flat.master.abs().max() if compress else 1e-5
    assert (r0 - eng.flat.master).abs().max() < tol


# ---------------------------------------------------------------------------
# per-rank ZeRO-1 optimizer shards in checkpoints: resume == uninterrupted
# ---------------------------------------------------------------------------
def _ckpt_worker(rank, world, port, q, path):
    ctx = _init(rank, world, port)
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(128)

    def batch(step):
        sl = slice(rank * 8 + step * 16, rank * 8 + step * 16 + 8)
        return torch.from_numpy(x[sl]), torch.from_numpy(y[sl])
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), Adam(lr=0.02), ctx=ctx, sharded=True, bucket_mb=0.0003)
    for s in range(3):
        eng.train_step(*batch(s))
    eng.set_checkpoint(path)
    eng.save_checkpoint()
    for s in range(3, 6):
        eng.train_step(*batch(s))
    eng.sync.sync_master()
    a = eng.flat.master.detach().numpy().copy()
    files = sorted(os.listdir(path))
    # a fresh engine (different init) resumes from the checkpoint
    eng2 = TrainingEngine(_mlp(seed=7), MeanSquaredError(), Adam(lr=0.02), ctx=ctx, sharded=True, bucket_mb=0.0003)
    eng2.set_checkpoint(path)
    eng2.load_checkpoint(eng2.latest_checkpoint())
    for s in range(3, 6):
        eng2.train_step(*batch(s))
    eng2.sync.sync_master()
    q.put((rank, (a, eng2.flat.master.detach().numpy().copy(), files)))
    ctx.stop()


def test_zero1_checkpoint_saves_every_rank_shard(tmp_path):
    res = _run(_ckpt_worker, str(tmp_path / "ck"))
    for r in (0, 1):
        a, b, files = res[r]
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-6)
    files = res[0][2]
    assert "optimMethod-Adam.rank0" in files and "optimMethod-Adam.rank1" in files and "model" in files


# ---------------------------------------------------------------------------
# a local failure on ONE rank: all ranks agree and reload together (no hang)
# ---------------------------------------------------------------------------
def _fail_worker(rank, world, port, q, path):
    ctx = _init(rank, world, port, ZOO_FAULT_INJECT_STEP=5, ZOO_FAULT_INJECT_RANK=1)
    from zoo.common import triggers as T
    from zoo.feature.common import FeatureSet
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(128)
    xs, ys = x[rank::2], y[rank::2]
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), SGD(learningrate=0.05), ctx=ctx, bucket_mb=0.0003)
    eng.set_checkpoint(path, T.SeveralIteration(2))
    eng.fit(FeatureSet.from_ndarrays(xs, ys, 8), end_trigger=T.MaxIteration(12), log_every=3)
    q.put((rank, (eng.flat.master.detach().numpy().copy(), eng._fault_fired, eng.state["neval"])))
    ctx.stop()


def test_failure_on_one_rank_is_agreed_and_retried(tmp_path):
    res = _run(_fail_worker, str(tmp_path / "ck"))
    (m0, f0, n0), (m1, f1, n1) = res[0], res[1]
    assert f1 and not f0
    assert n0 == n1 >= 12
    np.testing.assert_allclose(m0, m1, rtol=0, atol=1e-6)


# ---------------------------------------------------------------------------
# tensor parallelism through the engine: shards are not averaged across TP ranks
# ---------------------------------------------------------------------------
def _tp_worker(rank, world, port, q):
    ctx = _init(rank, world, port)
    from zoo.parallel.tensor_parallel import ParallelMLP
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    g = torch.Generator().manual_seed(3)
    w1, b1 = torch.randn(16, 6, generator=g) * 0.3, torch.randn(16, generator=g) * 0.1
    w2, b2 = torch.randn(6, 16, generator=g) * 0.3, torch.randn(6, generator=g) * 0.1
    mlp = ParallelMLP(6, 16, activation="relu", fc1=(w1, b1), fc2=(w2, b2))
    eng = TrainingEngine(mlp, MeanSquaredError(), SGD(learningrate=0.1), ctx=ctx)
    assert eng.sync.world == 1  # DP group: this rank alone (TP spans the world)
    x = torch.randn(8, 6, generator=g)
    y = torch.randn(8, 6, generator=g)
    for _ in range(3):
        eng.train_step(x, y)
    q.put((rank, (mlp.fc1.weight.detach().numpy().copy(), mlp.fc2.weight.detach().numpy().copy(),
                  mlp.fc2.bias.detach().numpy().copy())))
    ctx.stop()


def test_tensor_parallel_mlp_trains_through_engine():
    res = _run(_tp_worker)
    g = torch.Generator().manual_seed(3)
    w1, b1 = torch.randn(16, 6, generator=g) * 0.3, torch.randn(16, generator=g) * 0.1
    w2, b2 = torch.randn(6, 16, generator=g) * 0.3, torch.randn(6, generator=g) * 0.1
    x = torch.randn(8, 6, generator=g)
    y = torch.randn(8, 6, generator=g)
    full = nn.Sequential(nn.Linear(6, 16), nn.ReLU(), nn.Linear(16, 6))
    with torch.no_grad():
        full[0].weight.copy_(w1); full[0].bias.copy_(b1); full[2].weight.copy_(w2); full[2].bias.copy_(b2)
    opt = torch.optim.SGD(full.parameters(), lr=0.1)
    for _ in range(3):
        opt.zero_grad()
        ((full(x) - y) ** 2).mean().backward()
        opt.step()
    fc1 = np.concatenate([res[0][0], res[1][0]], 0)
    fc2 = np.concatenate([res[0][1], res[1][1]], 1)
    np.testing.assert_allclose(fc1, full[0].weight.detach().numpy(), atol=1e-5)
    np.testing.assert_allclose(fc2, full[2].weight.detach().numpy(), atol=1e-5)
    np.testing.assert_allclose(res[0][2], full[2].bias.detach().numpy(), atol=1e-5)


# ---------------------------------------------------------------------------
# row-sparse embedding-gradient sync (NCF at DP): equals the dense all-reduce
# ---------------------------------------------------------------------------
def _ncf_worker(rank, world, port, q, sparse, compress=""):
    ctx = _init(rank, world, port, ZOO_GRAD_COMPRESSION=compress)
    from zoo.models.recommendation.neuralcf import NeuralCF
    from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine
    torch.manual_seed(0)
    m = NeuralCF(500, 300, 5, user_embed=8, item_embed=8, hidden_layers=(16, 8), mf_embed=8,
                 row_sparse_sync=sparse)
    eng = TrainingEngine(m, SparseCategoricalCrossEntropy(), Adam(lr=0.01), ctx=ctx, bucket_mb=0.001)
    r = np.random.RandomState(100 + rank)
    for step in range(3):
        x = np.stack([r.randint(1, 60, 32), r.randint(1, 40, 32)], 1).astype(np.float32)
        y = r.randint(0, 5, 32).astype(np.int64)
        eng.train_step(torch.from_numpy(x), torch.from_numpy(y))
    nb = sum(1 for b in eng.sync.buckets if b.sparse)
    q.put((rank, (eng.flat.master.detach().numpy().copy(), nb, getattr(eng.sync, "sparse_rows", 0))))
    ctx.stop()


@pytest.mark.parametrize("compress", ["", "bf16"])
def test_row_sparse_embedding_sync_matches_dense_allreduce(compress):
    """fp32 wire, and the 16-bit wire (union rows packed to bf16, fp32 chunk sums, bf16 gather)
    against the dense bucket protocol on the same wire."""
    dense = _run(_ncf_worker, False, compress)
    sparse = _run(_ncf_worker, True, compress)
    for rk in (0, 1):
        assert np.allclose(dense[rk][0], sparse[rk][0], atol=1e-6), "row-sparse sync differs from dense"
    assert np.allclose(sparse[0][0], sparse[1][0], atol=1e-7), "ranks diverged"
    assert dense[0][1] == 0 and sparse[0][1] == 4        # four tables, one bucket each
    rows = sparse[0][2]
    assert 0 < rows < 3 * (2 * 501 + 2 * 301)            # only the looked-up union moved


# ---------------------------------------------------------------------------
# round 3: bucket launch order = calibrated readiness order, also for a zombie rank
# ---------------------------------------------------------------------------
class _OutOfOrder(nn.Module):
    """Registration order a, b, c; forward uses b first, then a, then c -> backward produces
    c, a, b: the flat layout (reverse registration: c, b, a) is NOT the readiness order."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = nn.Linear(8, 8)
        self.b = nn.Linear(6, 8)
        self.c = nn.Linear(8, 1)
        self.fail = False

    def forward(self, x):
        h = torch.tanh(self.b(x))
        h = torch.tanh(self.a(h))
        if self.fail:   # fails in backward, after c's gradient is produced
            h = _Boom.apply(h)
        return self.c(h)


class _Boom(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        raise RuntimeError("injected backward failure")


def _order_worker(rank, world, port, q):
    ctx = _init(rank, world, port)
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    m = _OutOfOrder()
    eng = TrainingEngine(m, MeanSquaredError(), SGD(learningrate=0.05), ctx=ctx, bucket_mb=1e-6)
    x, y = _toy(16)
    x, y = torch.from_numpy(x), torch.from_numpy(y)
    logs = []
    fin = eng.sync.finish

    def finish():
        fin()
        logs.append(list(eng.sync.launch_log))
    eng.sync.finish = finish
    for step in range(4):
        m.fail = (rank == 1 and step == 2)
        eng.train_step(x, y)
    q.put((rank, (logs, list(eng.sync.order), [b.params for b in eng.sync.buckets],
                  [id(p) for p in (m.c.weight, m.c.bias, m.a.weight, m.a.bias, m.b.weight, m.b.bias)],
                  eng._local_failure is not None)))
    ctx.stop()


def test_bucket_order_follows_readiness_and_zombie_replays_it():
    res = _run(_order_worker)
    logs0, order0, bparams, pids, _ = res[0]
    logs1, order1, _, _, zombie1 = res[1]
    assert zombie1 and order0 == order1
    # one parameter per bucket; readiness by layer = c, then a, then b (flat layout: c, b, a)
    layer_of = {pid: "ccaabb"[i] for i, pid in enumerate(pids)}
    assert [layer_of[bparams[i][0]] for i in order0] == list("ccaabb")
    assert order0 != sorted(order0)
    for s in range(1, 4):   # every later step (the zombie's step 2 included) launches in that order
        assert logs0[s] == order0 and logs1[s] == order0


# ---------------------------------------------------------------------------
# round 4: row-sparse capacity decisions are collective
# ---------------------------------------------------------------------------
def _ncf_var_worker(rank, world, port, q, sparse, users):
    ctx = _init(rank, world, port)
    from zoo.models.recommendation.neuralcf import NeuralCF
    from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine
    torch.manual_seed(0)
    m = NeuralCF(users, 300, 5, user_embed=8, item_embed=8, hidden_layers=(16, 8), mf_embed=8,
                 row_sparse_sync=sparse)
    eng = TrainingEngine(m, SparseCategoricalCrossEntropy(), Adam(lr=0.01), ctx=ctx, bucket_mb=0.001)
    r = np.random.RandomState(100 + rank)
    for step in range(3):
        # rank 1 looks up MORE ids than in the calibration step at step 2 (variable batch)
        n = 32 if not (rank == 1 and step == 2) else 96
        x = np.stack([r.randint(1, 60, n), r.randint(1, 40, n)], 1).astype(np.float32)
        y = r.randint(0, 5, n).astype(np.int64)
        eng.train_step(torch.from_numpy(x), torch.from_numpy(y))
    q.put((rank, (eng.flat.master.detach().numpy().copy(), getattr(eng.sync, "sparse_rows", 0))))
    ctx.stop()


def test_row_sparse_overflow_falls_back_together():
    """One rank exceeding the agreed lookup count must not raise or hang: the flag travels in the
    mask all-reduce and every rank reduces densely for that step -> equals the dense run."""
    dense = _run(_ncf_var_worker, False, 500)
    sparse = _run(_ncf_var_worker, True, 500)
    for rk in (0, 1):
        assert np.allclose(dense[rk][0], sparse[rk][0], atol=1e-6)
    assert np.allclose(sparse[0][0], sparse[1][0], atol=1e-7)


def test_row_sparse_picks_dense_when_union_covers_half_the_table():
    """Capacity = world * ids-per-step >= V/2: the mask + rows protocol would move more than the
    dense table, so the table is all-reduced densely (no mask all-reduce, no sparse rows)."""
    sparse = _run(_ncf_var_worker, True, 100)    # 2 ranks x 32 ids >= 101/2 for the user tables
    dense = _run(_ncf_var_worker, False, 100)
    for rk in (0, 1):
        assert np.allclose(dense[rk][0], sparse[rk][0], atol=1e-6)


# ---------------------------------------------------------------------------
# 4 ranks through the engine's bucketed all-reduce and ZeRO-1 paths
# ---------------------------------------------------------------------------
def _dp4_worker(rank, world, port, q, sharded, compress):
    ctx = _init(rank, world, port, ZOO_GRAD_COMPRESSION=compress)
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(96)
    per = 16 // world
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9), ctx=ctx,
                         sharded=sharded, bucket_mb=0.0003)
    nb = len(eng.sync.buckets)
    for step in range(5):
        sl = slice(step * 16 + rank * per, step * 16 + rank * per + per)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    eng.sync.sync_master()
    q.put((rank, (eng.flat.master.detach().numpy().copy(), nb, eng.sync.world)))
    ctx.stop()


@pytest.mark.parametrize("sharded,compress", [(False, ""), (False, "bf16"), (True, ""), (True, "bf16")])
def test_four_ranks_bucketed_and_zero1_match_single_process(sharded, compress):
    res = _run(_dp4_worker, sharded, compress, world=4)
    ws = [torch.from_numpy(res[r][0]) for r in range(4)]
    assert all(res[r][1] > 1 and res[r][2] == 4 for r in range(4)), "expected several buckets over 4 ranks"
    for w in ws[1:]:
        assert torch.allclose(ws[0], w, atol=1e-6), "ranks diverged"
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    x, y = _toy(96)
    eng = TrainingEngine(_mlp(seed=0), MeanSquaredError(), SGD(learningrate=0.1, momentum=0.9))
    for step in range(5):
        sl = slice(step * 16, step * 16 + 16)
        eng.train_step(torch.from_numpy(x[sl]), torch.from_numpy(y[sl]))
    tol = 2e-2 * eng.flat.master.abs().max() if compress else 1e-5
    assert (ws[0] - eng.flat.master).abs().max() < tol


# ---------------------------------------------------------------------------
# NNEstimator on per-rank DataFrame partitions (bench.py --input featureset)
# ---------------------------------------------------------------------------
def _local_part_worker(rank, world, port, q, n_local):
    ctx = _init(rank, world, port)
    import pandas as pd
    from zoo.common import triggers as T
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.nnframes.nn_classifier import NNEstimator
    x, y = _toy(64)
    xs, ys = x[rank::world][:n_local[rank]], y[rank::world][:n_local[rank]]
    df = pd.DataFrame({"features": list(xs), "label": list(ys)})
    est = NNEstimator(_mlp(seed=0), MeanSquaredError(), [6], [1]).setBatchSize(8).setLocalPartition(True)
    est.setOptimMethod(SGD(learningrate=0.1)).setEndWhen(T.MaxEpoch(3))
    try:
        est.fit(df)
    except ValueError as e:
        q.put((rank, ("error", str(e))))
        ctx.stop()
        return
    eng = est.engine
    q.put((rank, ("ok", eng.flat.master.detach().numpy().copy(), eng.state["neval"] - 1)))
    ctx.stop()


def test_nnestimator_local_partitions_train_in_lockstep():
    res = _run(_local_part_worker, (32, 32))
    (s0, m0, it0), (s1, m1, it1) = res[0], res[1]
    assert s0 == s1 == "ok"
    assert it0 == it1 == 3 * 32 // 4      # per-rank batch = 8 / 2 ranks, 3 epochs of 32 local rows
    np.testing.assert_allclose(m0, m1, rtol=0, atol=1e-6)


def test_nnestimator_local_partitions_must_be_equal():
    res = _run(_local_part_worker, (32, 24))
    assert res[0][0] == res[1][0] == "error" and "equal partitions" in res[0][1]
