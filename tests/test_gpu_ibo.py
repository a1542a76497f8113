"""In-backward optimizer (GradSync.enable_ibo: each bucket's update issued on the weight-gradient
side stream as soon as its gradients are final) against the plain end-of-step update: the same
training trajectory and the same final weights, for SGD-momentum on a ResNet and
AdamWeightDecay on a BERT stack, with small buckets so many updates overlap the backward."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(model, crit, optim, xs, y, steps, ibo, monkeypatch, bucket_mb=0.25):
    """Deterministic kernels (ordered statistics / split-K folds): a random-init network in
    training mode amplifies fp32-atomic reordering into visible loss differences, which would
    hide what this test compares."""
    from zoo.ops import native
    from zoo.pipeline.engine import TrainingEngine
    monkeypatch.setenv("ZOO_OPTIM_IN_BWD", "1" if ibo else "0")
    eng = TrainingEngine(model, crit, optim, bucket_mb=bucket_mb, hip_graph=False)
    assert eng.ibo == ibo
    native().set_deterministic(True)
    try:
        losses = [float(eng.train_step(xs, y).float().item()) for _ in range(steps)]
        torch.cuda.synchronize()
    finally:
        native().set_deterministic(False)
    if ibo:
        assert eng.sync.ibo_steps == steps and len(eng.sync.buckets) > 4
    w = eng.flat.master.detach().clone()
    return losses, w


def test_ibo_resnet_sgd_matches_end_of_step_update(gpu, monkeypatch):
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import resnet50
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    init_nncontext("ibo")
    torch.manual_seed(0)
    m = resnet50(num_classes=10)
    x = torch.randn(16, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (16,), device=gpu)
    runs = {}
    for ibo in (False, True):
        runs[ibo] = _train(copy.deepcopy(m), softmax_cross_entropy, SGD(learningrate=0.01, momentum=0.9), x, y, 6,
                           ibo, monkeypatch)
    (l0, w0), (l1, w1) = runs[False], runs[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (l0, l1)
    assert ((w1 - w0).norm() / w0.norm()).item() < 1e-5


def test_ibo_bert_adamw_matches_end_of_step_update(gpu, monkeypatch):
    import torch.nn as nn
    from zoo.common.nncontext import init_nncontext
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.layers import BERT
    from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
    init_nncontext("ibo-bert")
    torch.manual_seed(1)

    class Cls(nn.Module):
        def __init__(self):
            super().__init__()
            self.bert = BERT(vocab=500, hidden_size=256, n_block=2, n_head=4, max_position_len=64,
                             intermediate_size=1024, hidden_drop=0.0, attn_drop=0.0, output_all_block=False)
            self.fc = nn.Linear(256, 3)

        def forward(self, xs):
            return self.fc(self.bert(xs)[1].float())

    m = Cls()
    B, L = 32, 64
    xs = [torch.randint(0, 500, (B, L), device=gpu), torch.zeros(B, L, dtype=torch.long, device=gpu),
          torch.arange(L, device=gpu).repeat(B, 1), torch.ones(B, L, device=gpu)]
    y = torch.randint(0, 3, (B,), device=gpu)
    runs = {}
    for ibo in (False, True):
        runs[ibo] = _train(copy.deepcopy(m), softmax_cross_entropy, AdamWeightDecay(lr=1e-4), xs, y, 6, ibo,
                           monkeypatch, bucket_mb=0.5)
    (l0, w0), (l1, w1) = runs[False], runs[True]
    for a, b in zip(l0, l1):
        # (the embedding / attention backward keep fp32 atomics even in deterministic mode)
        assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (l0, l1)
    assert ((w1 - w0).norm() / w0.norm()).item() < 1e-4


class _SharedLoop(torch.nn.Module):
    """One native Dense layer applied ``uses[t]`` times in step t: every application's backward
    writes its weight gradient straight into the flat slot and counts as one contribution."""

    def __init__(self, uses):
        super().__init__()
        from zoo.ops import linear
        self._linear = linear
        self.w_in = torch.nn.Parameter(torch.randn(64, 32) * 0.1)
        self.w_mid = torch.nn.Parameter(torch.randn(64, 64) * 0.1)
        self.w_sh = torch.nn.Parameter(torch.randn(64, 64) * 0.1)
        self.b_sh = torch.nn.Parameter(torch.zeros(64))
        self.w_out = torch.nn.Parameter(torch.randn(8, 64) * 0.1)
        self.uses, self.t = list(uses), 0

    def forward(self, x):
        h = self._linear(x, self.w_in, None, act="relu")
        h = self._linear(h, self.w_mid, None, act="relu")
        k = self.uses[self.t % len(self.uses)]
        self.t += 1
        for _ in range(k):
            h = self._linear(h, self.w_sh, self.b_sh, act="relu")
        return self._linear(h, self.w_out, None).float()


def _shared_run(uses, ibo, monkeypatch, gpu, steps):
    from zoo.common.nncontext import init_nncontext
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    init_nncontext("ibo-shared")
    torch.manual_seed(3)
    m = _SharedLoop(uses)
    x = torch.randn(256, 32, device=gpu)
    y = torch.randint(0, 8, (256,), device=gpu)
    return _train(m, softmax_cross_entropy, SGD(learningrate=0.05, momentum=0.9), x, y, steps, ibo, monkeypatch,
                  bucket_mb=0.001), m


def test_ibo_variable_shared_layer_matches_end_of_step(gpu, monkeypatch):
    """Counts that differ between the two calibration steps keep the shared layer's bucket on
    the end-of-step update: the run equals ZOO_OPTIM_IN_BWD=0."""
    uses = [1, 2, 1, 3, 2, 2, 1, 3]
    (l0, w0), _ = _shared_run(uses, False, monkeypatch, gpu, 8)
    (l1, w1), _ = _shared_run(uses, True, monkeypatch, gpu, 8)
    for a, b in zip(l0, l1):
        assert abs(a - b) < 1e-5 * max(1.0, abs(b)), (l0, l1)
    assert ((w1 - w0).norm() / w0.norm()).item() < 1e-6


def test_ibo_late_contribution_degrades_without_raising(gpu, monkeypatch, caplog):
    """A count that grows AFTER calibration (2, 2, then 3 uses): the step completes, a warning
    is logged, the bucket moves to the end-of-step update for good, the late contribution is
    applied with the next update (not dropped), and the steps before the surprise match the
    end-of-step run exactly."""
    import logging
    uses = [2, 2, 2, 3, 2, 2]
    (l0, w0), _ = _shared_run(uses, False, monkeypatch, gpu, 6)
    with caplog.at_level(logging.WARNING, logger="zoo"):
        (l1, w1), _ = _shared_run(uses, True, monkeypatch, gpu, 6)
    assert any("in-backward optimizer" in r.getMessage() for r in caplog.records)
    for a, b in zip(l0[:4], l1[:4]):
        assert abs(a - b) < 1e-5 * max(1.0, abs(b)), (l0, l1)
    assert all(abs(v) < 1e3 for v in l1) and torch.isfinite(w1).all()
    assert ((w1 - w0).norm() / w0.norm()).item() < 0.05


def _bert_cls(gpu, drop, attn_drop=None):
    import torch.nn as nn
    from zoo.pipeline.api.keras.layers import BERT

    class Cls(nn.Module):
        def __init__(self):
            super().__init__()
            self.bert = BERT(vocab=500, hidden_size=256, n_block=2, n_head=4, max_position_len=64,
                             intermediate_size=1024, hidden_drop=drop,
                             attn_drop=drop if attn_drop is None else attn_drop, output_all_block=False)
            self.fc = nn.Linear(256, 3)

        def forward(self, xs):
            return self.fc(self.bert(xs)[1].float())
    B, L = 32, 64
    xs = [torch.randint(0, 500, (B, L), device=gpu), torch.zeros(B, L, dtype=torch.long, device=gpu),
          torch.arange(L, device=gpu).repeat(B, 1), torch.ones(B, L, device=gpu)]
    y = torch.randint(0, 3, (B,), device=gpu)
    return Cls(), xs, y


def test_graph_captured_ibo_matches_eager(gpu, monkeypatch):
    """BERT training with the forward, backward AND the in-backward AdamW updates captured in one
    hipGraph (learning rate / bias corrections read from device memory, staged before every
    replay) follows the eager end-of-step run within the bars of the eager IBO test."""
    from zoo.common.nncontext import init_nncontext
    from zoo.ops import native, softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("ibo-graph")
    torch.manual_seed(1)
    m, xs, y = _bert_cls(gpu, 0.0)
    runs = {}
    for graph in (False, True):
        monkeypatch.setenv("ZOO_OPTIM_IN_BWD", "1" if graph else "0")
        monkeypatch.setenv("ZOO_OPTIM_IN_BWD_GRAPH", "1")
        # total / warmup: the learning rate changes every step, so a baked-in rate would show
        eng = TrainingEngine(copy.deepcopy(m), softmax_cross_entropy,
                             AdamWeightDecay(lr=1e-4, warmup_portion=0.3, total=10), bucket_mb=0.5, hip_graph=graph)
        assert eng.ibo == graph
        native().set_deterministic(True)
        try:
            losses = [float(eng.train_step(xs, y).float().item()) for _ in range(7)]
            torch.cuda.synchronize()
        finally:
            native().set_deterministic(False)
        if graph:
            assert len(eng._graphs) == 1 and eng.sync.ibo_steps == 7
            assert len(next(iter(eng._graphs.values()))[4]) > 0     # in-backward updates inside the graph
        runs[graph] = (losses, eng.flat.master.detach().clone())
    (l0, w0), (l1, w1) = runs[False], runs[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (l0, l1)
    assert ((w1 - w0).norm() / w0.norm()).item() < 1e-4


def test_graph_replay_draws_fresh_dropout_masks(gpu):
    """Dropout inside a captured step: the seeds baked into the graph are xored with a device
    offset restaged every step, so replays of the SAME batch with frozen weights (lr 0) give
    different losses; with the offset held fixed they repeat exactly."""
    from zoo.common.nncontext import init_nncontext
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("graph-dropout")
    torch.manual_seed(2)
    m, xs, y = _bert_cls(gpu, 0.1)
    eng = TrainingEngine(m, softmax_cross_entropy, AdamWeightDecay(lr=0.0, weight_decay=0.0), hip_graph=True)
    losses = [float(eng.train_step(xs, y).float().item()) for _ in range(6)]
    assert len(eng._graphs) == 1
    replayed = losses[2:]
    assert len(set(round(v, 6) for v in replayed)) == len(replayed), losses
    eng._seed_rng.getrandbits = lambda k: 12345     # a frozen offset: identical masks on every replay
    frozen = [float(eng.train_step(xs, y).float().item()) for _ in range(3)]
    assert max(frozen) - min(frozen) < 1e-6, frozen


def test_graph_replay_attention_only_dropout_is_fresh(gpu):
    """Attention-probability dropout alone (hidden dropout 0): the fused attention kernels read
    the device seed offset, so the capture must mark it used and every replay draws new masks."""
    from zoo.common.nncontext import init_nncontext
    from zoo.ops import softmax_cross_entropy
    from zoo.ops.devscalar import seed_offset_used
    from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("graph-attn-dropout")
    torch.manual_seed(4)
    m, xs, y = _bert_cls(gpu, 0.0, attn_drop=0.2)
    eng = TrainingEngine(m, softmax_cross_entropy, AdamWeightDecay(lr=0.0, weight_decay=0.0), hip_graph=True)
    losses = [float(eng.train_step(xs, y).float().item()) for _ in range(6)]
    assert len(eng._graphs) == 1 and seed_offset_used(eng.device)
    replayed = losses[2:]
    assert len(set(round(v, 6) for v in replayed)) == len(replayed), losses


def test_clipping_after_capture_recaptures_without_inbwd_updates(gpu, monkeypatch):
    """A step captured WITH the in-backward updates must not be replayed once clipping is set
    (the captured updates are unclipped and step() would update the buckets a second time):
    the engine drops the graphs and recaptures a step without the updates."""
    from zoo.common.nncontext import init_nncontext
    from zoo.ops import softmax_cross_entropy
    from zoo.parallel.ddp import global_norm_clip
    from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
    from zoo.pipeline.engine import TrainingEngine
    monkeypatch.setenv("ZOO_OPTIM_IN_BWD", "1")
    monkeypatch.setenv("ZOO_OPTIM_IN_BWD_GRAPH", "1")
    init_nncontext("ibo-graph-clip")
    torch.manual_seed(5)
    m, xs, y = _bert_cls(gpu, 0.0)
    eng = TrainingEngine(m, softmax_cross_entropy, AdamWeightDecay(lr=1e-4), bucket_mb=0.5, hip_graph=True)
    assert eng.ibo
    for _ in range(4):
        eng.train_step(xs, y)
    assert len(eng._graphs) == 1 and len(next(iter(eng._graphs.values()))[4]) > 0
    eng.clip = global_norm_clip(1.0)
    eng.train_step(xs, y)
    assert not eng.ibo and not eng._graphs
    losses = [float(eng.train_step(xs, y).float().item()) for _ in range(4)]
    assert len(eng._graphs) == 1 and len(next(iter(eng._graphs.values()))[4]) == 0
    assert all(v == v and abs(v) < 1e3 for v in losses)
