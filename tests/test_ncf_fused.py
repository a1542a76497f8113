"""Fused NeuralCF kernels (csrc/kernels/ncf.hip, zoo.ops.ncf): the fp32 reference twin matches
the layer-by-layer Keras graph on the CPU; on the GPU the fused forward / backward match the
fp32 reference (probabilities, every parameter gradient) and train inside the engine.
Reference: NeuralCF.scala:45-138."""
import os

import pytest
import torch


def _model(users=50, items=40, mf=True, hidden=(40, 20, 10), classes=5, seed=0):
    from zoo.models.recommendation.neuralcf import NeuralCF
    torch.manual_seed(seed)
    m = NeuralCF(users, items, classes, user_embed=20, item_embed=20, hidden_layers=hidden, include_mf=mf,
                 mf_embed=20)
    # non-trivial biases (Dense initialises them to zero)
    with torch.no_grad():
        for d in m.__dict__["_ncf_parts"][4] + [m.__dict__["_ncf_parts"][5]]:
            d.bias.uniform_(-0.1, 0.1)
    return m


def _ref_args(m):
    eu, ei, emu, emi, dense, out = m.__dict__["_ncf_parts"]
    return [eu.embeddings, ei.embeddings, None if emu is None else emu.embeddings,
            None if emi is None else emi.embeddings, dense[0].weight, dense[0].bias, dense[1].weight,
            dense[1].bias, dense[2].weight, dense[2].bias, out.weight, out.bias]


def _ids(n, users, items, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.stack([torch.randint(0, users + 1, (n,), generator=g),
                        torch.randint(0, items + 1, (n,), generator=g)], 1)


@pytest.mark.parametrize("mf", [True, False])
def test_reference_matches_keras_graph(mf):
    from zoo.ops.ncf import ncf_reference
    m = _model(mf=mf).eval()
    x = _ids(64, 50, 40)
    with torch.no_grad():
        ref = ncf_reference(x, *_ref_args(m))
        out = m(x.float())
    torch.testing.assert_close(out.float(), ref, rtol=1e-5, atol=1e-6)


def test_fused_path_only_on_gpu_and_supported_widths():
    m = _model()
    x = _ids(8, 50, 40)
    assert m._fused_dims(x) is None                    # CPU tensor: layer graph
    m2 = _model(hidden=(40, 20))
    assert m2._fused_dims(x) is None                   # not three hidden layers


gpu_mark = pytest.mark.gpu


def _grads(m):
    return {n: (p.grad.detach().float().cpu().clone() if p.grad is not None else None)
            for n, p in m.named_parameters()}


@gpu_mark
@pytest.mark.parametrize("mf,B", [(True, 1000), (False, 513), (True, 65536)])
def test_fused_matches_fp32_reference(gpu, mf, B):
    import copy
    from torch.profiler import ProfilerActivity, profile
    from zoo.ops.ncf import ncf_reference
    m = _model(users=3000, items=2000, mf=mf)
    cpu = copy.deepcopy(m)
    g = copy.deepcopy(m).to(gpu)
    x = _ids(B, 3000, 2000)
    x[:3, 0] = torch.tensor([0, 3000, 7])             # boundary ids
    y = torch.randint(0, 5, (B,))
    assert g._fused_dims(x.to(gpu)) is not None
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        p = g(x.to(gpu))
        loss = torch.nn.functional.nll_loss(torch.log(p.clamp_min(1e-7)), y.to(gpu))
        loss.backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert any("ncf_kernel" in n for n in names), names[:10]
    assert not [n for n in names if "Cijk_" in n or "MIOpen" in n]
    pr = ncf_reference(x, *_ref_args(cpu))
    lr = torch.nn.functional.nll_loss(torch.log(pr.clamp_min(1e-7)), y)
    lr.backward()
    rel = ((p.float().cpu() - pr).norm() / pr.norm()).item()
    assert rel < 1e-2, rel
    # the emulated-bf16 twin: same model, rounded where the kernel stages through bf16
    emu = copy.deepcopy(m)
    pe = ncf_reference(x, *_ref_args(emu), bf16_stage=True)
    torch.nn.functional.nll_loss(torch.log(pe.clamp_min(1e-7)), y).backward()
    gg, gr, ge = _grads(g), _grads(cpu), _grads(emu)
    for n, a in gr.items():
        if a is None:
            continue
        b = gg[n]
        assert b is not None, n
        e = ((b - a).norm() / a.norm().clamp_min(1e-12)).item()
        e_emu = ((ge[n] - a).norm() / a.norm().clamp_min(1e-12)).item()
        # per-record bf16 staging noise (ReLU mask flips, rounded dZ rows) adds up as sqrt(B)
        # against a gradient that grows as B: at small batches the kernel is held to the
        # emulated-bf16 error, not to a fixed bound
        tol = 6e-2 if "embeddings" in n else 3e-2
        assert e < max(tol, 2.0 * e_emu) and e < 0.2, (n, e, e_emu)


@gpu_mark
def test_fused_trains_in_engine_like_layer_path(gpu, monkeypatch):
    """Three engine steps (flat fp32 master + bf16 copies, Adam, hipGraph) with the fused kernels
    follow the layer-by-layer graph's losses."""
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine
    init_nncontext("ncf-fused")
    x = _ids(4096, 3000, 2000).to(gpu)
    y = torch.randint(0, 5, (4096,), device=gpu)
    losses = {}
    import zoo.models.recommendation.neuralcf as ncf_mod
    for mode in ("1", "0"):
        monkeypatch.setattr(ncf_mod, "_NCF_FUSED", mode == "1")
        m = _model(users=3000, items=2000)
        eng = TrainingEngine(m, SparseCategoricalCrossEntropy(), Adam(lr=1e-2), hip_graph=True)
        losses[mode] = [float(eng.train_step(x, y).item()) for _ in range(6)]
    a, b = losses["1"], losses["0"]
    assert all(l == l for l in a), a
    assert a[-1] < a[0], a
    for u, v in zip(a, b):
        assert abs(u - v) < 2e-2 * max(1.0, abs(v)), (a, b)


def _nll_ref(p, y, ignore=-100, size_average=True):
    logp = torch.log(torch.clamp(p.float(), 1e-7, 1.0))
    return torch.nn.functional.nll_loss(logp, y, ignore_index=ignore, reduction="mean" if size_average else "sum")


def test_prob_nll_cpu_matches_formula():
    from zoo.ops import prob_nll
    torch.manual_seed(0)
    p = torch.softmax(torch.randn(33, 5), -1)
    y = torch.randint(0, 5, (33,))
    torch.testing.assert_close(prob_nll(p, y), _nll_ref(p, y))


@gpu_mark
@pytest.mark.parametrize("size_average", [True, False])
def test_prob_nll_native_loss_and_grad(gpu, size_average):
    from zoo.ops import prob_nll
    torch.manual_seed(0)
    p = torch.softmax(torch.randn(1000, 5), -1)
    p[0] = torch.tensor([0.0, 0.0, 0.0, 0.0, 1.0])          # clamped label probability
    y = torch.randint(0, 5, (1000,))
    y[0], y[5] = 1, 3
    y[7] = -1                                                # ignored with ignore_index=-1
    pc = p.clone().requires_grad_(True)
    lc = _nll_ref(pc, y, -1, size_average)
    lc.backward()
    pg = p.to(gpu).requires_grad_(True)
    lg = prob_nll(pg, y.to(gpu), 1e-7, -1, size_average)
    lg.backward()
    torch.testing.assert_close(lg.cpu(), lc, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(pg.grad.cpu(), pc.grad, rtol=1e-5, atol=1e-6)
