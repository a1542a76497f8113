"""Synthetic, learnable image-classification data for accuracy-style checks without datasets.

There is no network access for ImageNet or pretrained checkpoints, and a random-init network is a
poor judge of a lossy transform (int8 / fp8 inference): its logits barely depend on the input,
so the top-1 class flips on noise far below any real model's decision margins. This module
builds a task a network learns in a few dozen steps -- each class is a fixed smooth random
pattern, every sample is its class pattern under a random contrast / brightness / shift plus
noise -- and ``train_briefly`` fits a model to it, so quantized-vs-bf16 agreement is measured
on confident, input-dependent predictions (tools/quant_bench.py, tests/test_gpu_qconv.py).
"""
import torch
import torch.nn.functional as F


def class_templates(num_classes, hw, seed=0, device="cpu"):
    """[num_classes, 3, hw, hw] smooth random patterns (low-frequency noise, unit variance)."""
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(num_classes, 3, max(hw // 16, 2), max(hw // 16, 2), generator=g)
    t = F.interpolate(base, size=(hw, hw), mode="bilinear", align_corners=False)
    t = (t - t.mean((2, 3), keepdim=True)) / t.std((2, 3), keepdim=True).clamp_min(1e-6)
    return t.to(device)


def sample(templates, n, seed=1, noise=0.5):
    """n labelled samples: class pattern x contrast + brightness, rolled a few pixels, + noise."""
    g = torch.Generator().manual_seed(seed)
    C = templates.shape[0]
    y = torch.randint(0, C, (n,), generator=g)
    x = templates.cpu()[y]
    contrast = torch.rand(n, 1, 1, 1, generator=g) * 0.8 + 0.6
    bright = torch.randn(n, 1, 1, 1, generator=g) * 0.2
    x = x * contrast + bright
    sh = torch.randint(-3, 4, (2,), generator=g)
    x = torch.roll(x, (int(sh[0]), int(sh[1])), (2, 3))
    x = x + torch.randn(x.shape, generator=g) * noise
    return x.to(templates.device), y.to(templates.device)


def train_briefly(model, templates, steps=300, batch=32, lr=0.01, seed=2):
    """Fit ``model`` (a zoo image classifier, NCHW input) to the synthetic task with the
    framework's own training engine; returns the accuracy on a fresh batch. (ResNet-50 from
    scratch, batch 32 at 128x128: 300 steps at lr 0.01 reach 1.0; 80 steps at lr 0.05 diverge
    early and stay near chance -- scripts/r4/dbg_fail.sh sweep.)"""
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    eng = TrainingEngine(model, softmax_cross_entropy, SGD(learningrate=lr, momentum=0.9))
    for s in range(steps):
        x, y = sample(templates, batch, seed=seed * 100003 + s)
        eng.train_step(x, y)
    eng.flat.detach()          # parameters back to private storage (the engine is discarded)
    model.eval()
    x, y = sample(templates, 4 * batch, seed=seed * 7 + 999)
    with torch.no_grad():
        acc = (model(x).float().argmax(1) == y).float().mean().item()
    return acc


def input_sensitivity(ref):
    """Spread of a model's logits ACROSS inputs (mean over classes of the per-class std over the
    batch) relative to their mean magnitude: ~0 for a collapsed model that ignores its input, on
    which any agreement number is vacuous."""
    ref = ref.float()
    return (ref.std(0).mean() / ref.abs().mean().clamp_min(1e-12)).item()


def margin_agreement(out, ref, rel_margin=0.1):
    """Top-1 agreement over the samples whose reference top-1 / top-2 logit margin is at least
    ``rel_margin`` of that row's logit std (a near-tie flips on any rounding); returns
    (agreement, fraction of samples kept)."""
    out, ref = out.float(), ref.float()
    top2 = ref.topk(2, dim=1).values
    keep = (top2[:, 0] - top2[:, 1]) >= rel_margin * ref.std(1)
    if not bool(keep.any()):
        return float("nan"), 0.0
    agree = (out.argmax(1) == ref.argmax(1))[keep].float().mean().item()
    return agree, keep.float().mean().item()


def agreement(out, ref):
    """(top-1 agreement, mean per-sample cosine of mean-centred logits) of two logit batches."""
    out, ref = out.float(), ref.float()
    top1 = (out.argmax(1) == ref.argmax(1)).float().mean().item()
    a = out - out.mean(1, keepdim=True)
    b = ref - ref.mean(1, keepdim=True)
    cos = F.cosine_similarity(a, b, dim=1).mean().item()
    return top1, cos
