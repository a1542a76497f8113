"""HK10 sparse kernels (csrc/kernels/sparse.hip) against plain PyTorch fp32
references: embedding bag (dense-padded and CSR bags, sum/mean/sqrtn, per-id
weights, max-norm) and sparse linear (COO input), forward and backward, plus the
Keras SparseEmbedding / SparseDense layers and Wide&Deep on the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _torch_bag(table, ids, offsets, weights, combiner, max_norm):
    """oracle on torch.nn.functional.embedding_bag where it applies"""
    import torch.nn.functional as F
    mode = {"sum": "sum", "mean": "mean"}[combiner]
    return F.embedding_bag(ids, table, offsets, mode=mode, per_sample_weights=weights)


@pytest.mark.parametrize("D", [16, 64, 300, 7])
@pytest.mark.parametrize("combiner", ["sum", "mean", "sqrtn"])
def test_embedding_bag_dense_ids(gpu, D, combiner):
    from zoo.ops.sparse import embedding_bag, embedding_bag_ref
    torch.manual_seed(0)
    V, B, L = 500, 37, 9
    table = torch.randn(V, D, device=gpu, requires_grad=True)
    ids = torch.randint(-2, V, (B, L), device=gpu)
    ids[3] = -1                                  # an all-padding bag
    out = embedding_bag(table, ids, combiner=combiner)
    t2 = table.detach().clone().requires_grad_(True)
    ref = embedding_bag_ref(t2, ids, combiner=combiner)
    assert rel(out, ref) < 1e-5
    assert out[3].abs().max().item() == 0.0
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g)
    assert rel(table.grad, t2.grad) < 1e-5


@pytest.mark.parametrize("combiner", ["sum", "mean"])
def test_embedding_bag_csr_weighted_vs_torch(gpu, combiner):
    from zoo.ops.sparse import embedding_bag
    torch.manual_seed(1)
    V, D, B = 1000, 32, 64
    lens = torch.randint(0, 12, (B,))
    offsets = torch.zeros(B + 1, dtype=torch.long)
    offsets[1:] = lens.cumsum(0)
    ids = torch.randint(0, V, (int(offsets[-1]),), device=gpu)
    offsets = offsets.to(gpu)
    w = torch.rand(ids.numel(), device=gpu) + 0.1
    table = torch.randn(V, D, device=gpu, requires_grad=True)
    out = embedding_bag(table, ids, offsets, w, combiner)
    t2 = table.detach().clone().requires_grad_(True)
    if combiner == "sum":
        ref = _torch_bag(t2, ids, offsets[:-1], w, combiner, None)
    else:  # torch's mean ignores per-sample weights: weighted sum / sum of weights by hand
        s = _torch_bag(t2, ids, offsets[:-1], w, "sum", None)
        den = torch.zeros(B, device=gpu).index_add(0, torch.repeat_interleave(torch.arange(B, device=gpu),
                                                                             offsets[1:] - offsets[:-1]), w)
        ref = s / den.clamp_min(1e-12)[:, None]
    assert rel(out, ref) < 1e-5
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g)
    assert rel(table.grad, t2.grad) < 1e-5


def test_embedding_bag_max_norm(gpu):
    from zoo.ops.sparse import embedding_bag, embedding_bag_ref
    torch.manual_seed(2)
    table = (torch.randn(100, 24, device=gpu) * 3).requires_grad_(True)
    ids = torch.randint(0, 100, (16, 5), device=gpu)
    out = embedding_bag(table, ids, combiner="sqrtn", max_norm=2.0)
    t2 = table.detach().clone().requires_grad_(True)
    ref = embedding_bag_ref(t2, ids, combiner="sqrtn", max_norm=2.0)
    assert rel(out, ref) < 1e-5
    out.sum().backward()
    ref.sum().backward()
    assert rel(table.grad, t2.grad) < 1e-5


@pytest.mark.parametrize("O,IN", [(2, 5000), (5, 777), (130, 300)])
def test_sparse_linear_coo(gpu, O, IN):
    from zoo.ops.sparse import sparse_linear
    torch.manual_seed(3)
    B = 96
    dense = torch.zeros(B, IN, device=gpu)
    nz = torch.randint(0, IN, (B, 6), device=gpu)
    dense.scatter_(1, nz, torch.rand(B, 6, device=gpu) + 0.5)
    x = dense.to_sparse()
    w = (torch.randn(O, IN, device=gpu) * 0.1).requires_grad_(True)
    b = torch.randn(O, device=gpu, requires_grad=True)
    y = sparse_linear(x, w, b)
    w2 = w.detach().clone().requires_grad_(True)
    b2 = b.detach().clone().requires_grad_(True)
    ref = dense @ w2.t() + b2
    assert rel(y, ref) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    assert rel(w.grad, w2.grad) < 1e-5
    assert rel(b.grad, b2.grad) < 1e-5


def test_sparse_keras_layers_and_wide_and_deep_train_on_gpu(gpu):
    from zoo.models.recommendation.wide_and_deep import ColumnFeatureInfo, WideAndDeep
    from zoo.pipeline.api.keras.layers import SparseDense, SparseEmbedding
    torch.manual_seed(4)
    se = SparseEmbedding(200, 16, combiner="mean")
    se._ensure_built((None, 7))
    se = se.to(gpu)
    ids = torch.randint(-1, 200, (32, 7), device=gpu)
    out = se(ids)
    assert out.shape == (32, 16) and torch.isfinite(out).all()
    sd = SparseDense(4)
    sd._ensure_built((None, 1000))
    sd = sd.to(gpu)
    dense = (torch.rand(32, 1000, device=gpu) > 0.99).float()
    assert rel(sd(dense.to_sparse()), sd(dense)) < 1e-5
    # Wide&Deep (ml-20m shape, small MLP) trains through the engine on the native sparse path
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "analytics-zoo_amd", "tools"))
    from wnd_bench import build
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine
    model, xs, y = build(512, gpu, hidden=(64, 32))
    eng = TrainingEngine(model, ClassNLLCriterion(log_prob_as_input=False, zero_based_label=False), Adam(lr=1e-2))
    losses = [float(eng.train_step(xs, y)) for _ in range(15)]
    assert losses[-1] < losses[0], losses


@pytest.mark.gpu
def test_wnd_deep_input_and_head_match_torch(gpu):
    """Wide&Deep fused kernels (csrc/kernels/wnd.hip) vs the fp32 torch composition: the deep
    input row (indicator | two embedding lookups from float ids | continuous; out-of-range id
    -> zeros) forward + table gradients, and softmax(wide + bias + deep) forward + all three
    gradients (fp32 and bf16 deep tower)."""
    from zoo.ops.wnd import deep_input, wnd_head
    torch.manual_seed(9)
    B = 1000
    ind = (torch.rand(B, 23, device=gpu) > 0.8).float()
    cont = torch.rand(B, 1, device=gpu)
    t0 = torch.randn(301, 64, device=gpu, requires_grad=True)
    t1 = torch.randn(57, 16, device=gpu, requires_grad=True)
    ids = torch.stack([torch.randint(0, 301, (B,), device=gpu), torch.randint(0, 57, (B,), device=gpu)], 1).float()
    ids[3, 1] = 57                                        # out of range -> zero row, no gradient
    out = deep_input(ids, [("dense", ind), ("embed", t0, 0), ("embed", t1, 1), ("dense", cont)])
    assert out.dtype == torch.bfloat16 and out.shape == (B, 23 + 64 + 16 + 1)
    r0, r1 = t0.detach().clone().requires_grad_(True), t1.detach().clone().requires_grad_(True)
    i1 = ids[:, 1].long()
    e1 = r1[i1.clamp(max=56)] * (i1 < 57).float().unsqueeze(1)
    ref = torch.cat([ind, r0[ids[:, 0].long()], e1, cont], 1)
    assert rel(out.float(), ref) < 1e-2
    g = torch.randn(B, ref.shape[1], device=gpu)
    out.backward(g.bfloat16())
    ref.backward(g.bfloat16().float())
    assert rel(t0.grad, r0.grad) < 1e-4
    assert rel(t1.grad, r1.grad) < 1e-4
    for dd in (torch.float32, torch.bfloat16):
        wide = torch.randn(B, 5, device=gpu, requires_grad=True)
        deep = torch.randn(B, 5, device=gpu).to(dd).requires_grad_(True)
        bias = torch.randn(5, device=gpu, requires_grad=True)
        p = wnd_head(wide, deep, bias)
        wr, dr, br = (t.detach().float().clone().requires_grad_(True) for t in (wide, deep, bias))
        pr = torch.softmax(wr + br + dr, -1)
        assert rel(p, pr) < 1e-5
        gp = torch.randn(B, 5, device=gpu)
        p.backward(gp)
        pr.backward(gp)
        assert rel(wide.grad, wr.grad) < 1e-4
        assert rel(deep.grad.float(), dr.grad) < 1e-2
        assert rel(bias.grad, br.grad) < 1e-4
