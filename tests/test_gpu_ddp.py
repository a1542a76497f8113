"""The data-parallel engine's collective path on a real GPU: a world-size-1 RCCL
process group with ``force_comm`` runs the bucketed, comm-stream, event-ordered
path (all_reduce / reduce_scatter_tensor / all_to_all_single /
all_gather_into_tensor) and must reproduce the local (no-comm) step bit for bit
under the deterministic reduction mode."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_world1():
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zoo.common.nncontext import init_nncontext
    ctx = init_nncontext("ddp-test")
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
        created = True
    yield ctx
    if created:
        dist.destroy_process_group()


def _model():
    from zoo.models.image.resnet import Bottleneck, ResNet
    torch.manual_seed(3)
    return ResNet(Bottleneck, [1, 1, 1, 1], num_classes=16, width=16)


def _train(ctx, force, sharded=False, compress=None, steps=4):
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    old = (ctx.config.force_comm, ctx.config.grad_compression)
    ctx.config.force_comm, ctx.config.grad_compression = force, (compress or "") if compress != "default" else old[1]
    try:
        eng = TrainingEngine(_model(), softmax_cross_entropy, SGD(learningrate=0.05, momentum=0.9), ctx=ctx,
                             sharded=sharded, bucket_mb=0.05)
    finally:
        ctx.config.force_comm, ctx.config.grad_compression = old
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device="cuda", generator=g)
    y = torch.randint(0, 16, (8,), device="cuda", generator=g)
    early = []
    fin = eng.sync.finish

    def finish():
        early.append(sum(b.launched for b in eng.sync.buckets))
        fin()
    eng.sync.finish = finish
    losses = [eng.train_step(x, y).float().item() for _ in range(steps)]
    torch.cuda.synchronize()
    eng.sync.sync_master()
    return eng, losses, early


@pytest.mark.parametrize("sharded", [False, True])
def test_forced_comm_matches_local_bitwise(gpu, rccl_world1, sharded):
    from zoo.ops import deterministic, set_deterministic
    prev = deterministic()
    set_deterministic(True)
    try:
        e0, l0, _ = _train(rccl_world1, force=False)
        e1, l1, early = _train(rccl_world1, force=True, sharded=sharded)
    finally:
        set_deterministic(prev)
    assert e1.sync.comm and len(e1.sync.buckets) > 2
    assert early[0] == 0, "calibration step must not launch early"
    assert max(early[1:]) > 0, "no bucket overlapped with backward"
    assert l0 == l1
    assert torch.equal(e0.flat.bf16, e1.flat.bf16)
    assert torch.equal(e0.flat.master, e1.flat.master)


def test_forced_comm_bf16_wire_tracks_fp32(gpu, rccl_world1):
    e0, l0, _ = _train(rccl_world1, force=False)
    e1, l1, _ = _train(rccl_world1, force=True, compress="bf16")
    e2, l2, _ = _train(rccl_world1, force=True, sharded=True, compress="bf16")
    for a, b, c in zip(l0, l1, l2):
        assert abs(a - b) < 0.05 and abs(a - c) < 0.05
    for e in (e1, e2):  # bf16 gradient rounding: a small relative perturbation of the update
        d = (e0.flat.master - e.flat.master).norm() / e0.flat.master.norm()
        assert d.item() < 0.01


def test_default_wire_is_bf16_and_tracks_fp32(gpu, rccl_world1):
    """The config default ("auto") puts gradients on a bf16 wire with fp32 accumulation whenever
    GPU collectives run (BigDL's 16-bit gradient transfer), in both sync modes."""
    assert rccl_world1.config.grad_compression == "auto"
    e0, l0, _ = _train(rccl_world1, force=False)
    e1, l1, _ = _train(rccl_world1, force=True, compress="default")
    e2, l2, _ = _train(rccl_world1, force=True, sharded=True, compress="default")
    assert e0.sync.compress is None and e1.sync.compress == "bf16" and e2.sync.compress == "bf16"
    for a, b, c in zip(l0, l1, l2):
        assert abs(a - b) < 0.05 and abs(a - c) < 0.05
    for e in (e1, e2):
        d = (e0.flat.master - e.flat.master).norm() / e0.flat.master.norm()
        assert d.item() < 0.01


def test_zombie_finish_replays_the_recorded_bucket_order(gpu, rccl_world1):
    """Healthy steps launch buckets in the calibrated readiness order; a rank that failed
    part-way through backward (some buckets launched, the rest not) finishes in that same
    order, so its RCCL collective sequence matches the healthy ranks'."""
    eng, _, _ = _train(rccl_world1, force=True, steps=3)
    s = eng.sync
    assert s.order is not None and sorted(s.order) == list(range(len(s.buckets)))
    s.reset()
    for i in s.order[:2]:           # the zombie got this far before failing
        s._launch(s.buckets[i])
    s.wait_comm()
    eng.flat.grad.zero_()
    s.finish()
    assert s.launch_log == s.order
    torch.cuda.synchronize()
    s.reset()


def test_comm_stats_fields(gpu, rccl_world1):
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    ctx = rccl_world1
    old = ctx.config.force_comm
    ctx.config.force_comm = True
    try:
        eng = TrainingEngine(_model(), softmax_cross_entropy, SGD(learningrate=0.05), ctx=ctx, bucket_mb=0.05)
    finally:
        ctx.config.force_comm = old
    eng.sync.collect_stats = True
    x = torch.randn(8, 3, 64, 64, device="cuda")
    y = torch.randint(0, 16, (8,), device="cuda")
    for _ in range(3):
        eng.train_step(x, y)
    summ = eng.sync.comm_summary()
    assert summ["exposed_comm_ms_per_step"] >= 0.0
    assert len(summ["buckets"]) == len(eng.sync.buckets)
    assert all(b["ms"] >= 0 and b["bytes"] > 0 for b in summ["buckets"])


class _EmbMLP(torch.nn.Module):
    """An fp32 embedding table (compute_dtype=None: the lookup reads the fp32 master) feeding a
    plain torch Linear (fp32 weight read): no parameter here is read through a bf16 copy."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(5)
        self.table = torch.nn.Parameter(torch.randn(200, 16) * 0.3)
        self.fc = torch.nn.Linear(16, 4)

    def forward(self, idx):
        from zoo.ops.nn import embedding
        return self.fc(embedding(idx, self.table).mean(1))


def test_zero1_keeps_fp32_read_parameters_exact(gpu, rccl_world1):
    """ZeRO-1 gathers bf16 weights only for parameters a native kernel reads through the bf16
    copy; fp32-read tables and torch layers must train exactly as in all-reduce mode."""
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    ctx = rccl_world1
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    idx = torch.randint(0, 200, (32, 6), device="cuda", generator=g)
    y = torch.randn(32, 4, device="cuda", generator=g)
    masters = []
    for sharded in (False, True):
        old = (ctx.config.force_comm, ctx.config.grad_compression)
        ctx.config.force_comm, ctx.config.grad_compression = True, ""
        try:
            eng = TrainingEngine(_EmbMLP(), MeanSquaredError(), SGD(learningrate=0.5), ctx=ctx, sharded=sharded,
                                 bucket_mb=0.004)
        finally:
            ctx.config.force_comm, ctx.config.grad_compression = old
        for _ in range(3):
            eng.train_step(idx, y)
        torch.cuda.synchronize()
        masters.append(eng.flat.master.clone())   # what the layers read (no sync_master)
    assert not getattr(eng.model.table, "_zoo_bf16_read", False)
    assert torch.allclose(masters[0], masters[1], rtol=0, atol=1e-6), \
        (masters[0] - masters[1]).abs().max().item()
