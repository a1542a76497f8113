"""The C++ comm layer (csrc/comm.cpp, zoo/parallel/comm.py): RCCL communicators of our own,
bootstrapped through the torch.distributed group, collectives on the current stream. On the
one-GPU box the communicator has one rank: every collective is then an identity / copy, which
pins the plumbing (dtypes, sizes, streams, group fusion, channel config) and -- through the
engine -- that GradSync's bucket path over the native layer reproduces the local step bit for
bit, as the ProcessGroup path does (tests/test_gpu_ddp.py). Multi-rank behaviour is RCCL's."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_world1():
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zoo.common.nncontext import init_nncontext
    ctx = init_nncontext("comm-test")
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
        created = True
    yield ctx
    if created:
        dist.destroy_process_group()


@pytest.mark.parametrize("channels", [0, 8])
def test_native_collectives_world1(gpu, rccl_world1, channels):
    from zoo.parallel.comm import NativeComm
    c = NativeComm(None, channels=channels)
    try:
        assert (c.rank, c.world) == (0, 1)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for dt in (torch.float32, torch.bfloat16, torch.int32, torch.uint8):
                t = (torch.arange(1000, device=gpu) % 97).to(dt)
                ref = t.clone()
                c.all_reduce(t)
                assert torch.equal(t, ref)
                out = torch.empty_like(t)
                c.all_gather(out, t)
                assert torch.equal(out, ref)
                out.zero_()
                c.all_to_all(out, t)
                assert torch.equal(out, ref)
                out.zero_()
                c.reduce_scatter(out, t)
                assert torch.equal(out, ref)
                c.broadcast(t, 0)
                assert torch.equal(t, ref)
            a = torch.randn(4096, device=gpu)
            b = torch.randn(4096, device=gpu).to(torch.bfloat16)
            oa, ob = torch.empty_like(a), torch.empty_like(b)
            with c.fused():     # one fused launch group
                c.all_to_all(oa, a)
                c.all_gather(ob, b)
        s.synchronize()
        assert torch.equal(oa, a) and torch.equal(ob, b)
        t = torch.ones(8, device=gpu)
        c.all_reduce(t, "avg")
        assert torch.equal(t, torch.ones(8, device=gpu))
    finally:
        c.close()


@pytest.mark.parametrize("sharded", [False, True])
def test_engine_over_native_comm_matches_local_bitwise(gpu, rccl_world1, sharded):
    """Deterministic reductions: the engine with force_comm and comm="native" (GradSync's bucket
    collectives through the C++ layer) gives the local step's weights bit for bit."""
    from zoo.models.image.resnet import Bottleneck, ResNet
    from zoo.ops import deterministic, set_deterministic, softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    ctx = rccl_world1
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device="cuda", generator=g)
    y = torch.randint(0, 16, (8,), device="cuda", generator=g)

    def run(force, comm):
        old = (ctx.config.force_comm, ctx.config.comm, ctx.config.grad_compression)
        ctx.config.force_comm, ctx.config.comm, ctx.config.grad_compression = force, comm, ""
        try:
            torch.manual_seed(3)
            eng = TrainingEngine(ResNet(Bottleneck, [1, 1, 1, 1], num_classes=16, width=16), softmax_cross_entropy,
                                 SGD(learningrate=0.05, momentum=0.9), ctx=ctx, sharded=sharded, bucket_mb=0.05)
        finally:
            ctx.config.force_comm, ctx.config.comm, ctx.config.grad_compression = old
        losses = [eng.train_step(x, y).float().item() for _ in range(4)]
        torch.cuda.synchronize()
        eng.sync.sync_master()
        return eng, losses
    prev = deterministic()
    set_deterministic(True)
    try:
        e0, l0 = run(False, "torch")
        e1, l1 = run(True, "native")
    finally:
        set_deterministic(prev)
    assert e1.sync.ncomm is not None and len(e1.sync.buckets) > 2
    assert l0 == l1
    assert torch.equal(e0.flat.master, e1.flat.master)


def test_full_step_graph_over_native_comm_matches_eager_bitwise(gpu, rccl_world1):
    """with comm="native" and hip_graph the WHOLE data-parallel step -- forward,
    backward, the bucket collectives (RCCL, captured on the comm stream) and the optimizer
    update (device-scalar lr) -- is one graph replay, and in deterministic mode it reproduces the
    eager step over the same communicator bit for bit, with an lr schedule that changes every step."""
    from zoo.models.image.resnet import Bottleneck, ResNet
    from zoo.ops import deterministic, set_deterministic, softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD, Poly
    from zoo.pipeline.engine import TrainingEngine
    ctx = rccl_world1
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    x = torch.randn(8, 3, 64, 64, device="cuda", generator=g)
    y = torch.randint(0, 16, (8,), device="cuda", generator=g)

    def run(graph):
        old = (ctx.config.force_comm, ctx.config.comm, ctx.config.grad_compression)
        ctx.config.force_comm, ctx.config.comm, ctx.config.grad_compression = True, "native", "bf16"
        try:
            torch.manual_seed(3)
            eng = TrainingEngine(ResNet(Bottleneck, [1, 1, 1, 1], num_classes=16, width=16), softmax_cross_entropy,
                                 SGD(learningrate=0.05, momentum=0.9, learningrate_schedule=Poly(0.5, 20)),
                                 ctx=ctx, bucket_mb=0.05, hip_graph=graph)
        finally:
            ctx.config.force_comm, ctx.config.comm, ctx.config.grad_compression = old
        losses = [eng.train_step(x, y).float().item() for _ in range(7)]
        torch.cuda.synchronize()
        return eng, losses
    prev = deterministic()
    set_deterministic(True)
    try:
        e0, l0 = run(False)
        e1, l1 = run(True)
    finally:
        set_deterministic(prev)
    assert e1.full_graph and e1.sync.ncomm is not None and len(e1.sync.buckets) > 2
    assert len(e1._graphs) == 1 and next(iter(e1._graphs.values()))[5]   # collectives + update captured
    assert e1.optim.state["neval"] == e0.optim.state["neval"] == 8
    assert l0 == l1, (l0, l1)
    assert torch.equal(e0.flat.master, e1.flat.master)
