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
