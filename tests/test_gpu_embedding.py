"""Native embedding gather / scatter-add backward (csrc/kernels/nn_misc.hip) against
torch fp32: the LDS-privatised path for small tables (position / token-type rows hit by
thousands of tokens) and the run-merging path for large vocabularies, fp32 and bf16
gradients, padding ids and out-of-range ids (Zs LookupTable accGradParameters)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_grad(V, D, ids, dout, pad):
    g = torch.zeros(V, D, dtype=torch.float64, device=dout.device)
    keep = (ids >= 0) & (ids < V)
    if pad >= 0:
        keep &= ids != pad
    g.index_add_(0, ids[keep], dout.double()[keep])
    return g


@pytest.mark.parametrize("V,D,pattern", [
    (2, 768, "random"), (2, 768, "zeros"), (512, 768, "positions"), (100, 64, "random"),
    (30522, 768, "random"), (30522, 768, "runs"), (1000, 12, "random"),
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_embedding_bwd_matches_index_add(gpu, V, D, pattern, dtype):
    from zoo.ops import native
    if dtype == torch.bfloat16 and D % 8:
        pytest.skip("bf16 rows need 16-byte alignment")
    torch.manual_seed(0)
    B, L = 32, 128
    if pattern == "zeros":
        ids = torch.zeros(B, L, dtype=torch.long)
    elif pattern == "positions":
        ids = torch.arange(L).repeat(B, 1)
    elif pattern == "runs":
        ids = torch.randint(0, V, (B, L // 8)).repeat_interleave(8, dim=1)
    else:
        ids = torch.randint(0, V, (B, L))
    ids = ids.reshape(-1).to(gpu)
    ids[::97] = -1          # out of range -> skipped
    pad = 1 if V > 1 else -1
    dout = torch.randn(ids.numel(), D, device=gpu).to(dtype)
    g = torch.zeros(V, D, device=gpu)
    native().embedding_bwd(dout.contiguous(), ids, g, pad, 0.5)
    ref = 0.5 * _ref_grad(V, D, ids, dout.float(), pad)
    err = ((g.double() - ref).norm() / ref.norm().clamp_min(1e-12)).item()
    assert err < 1e-5, err
    if pad >= 0:
        assert g[pad].abs().max().item() == 0.0


def test_bert_style_embeddings_train_step(gpu):
    """word + position + token-type lookups through zoo.ops.embedding: table grads vs torch"""
    from zoo.ops.nn import embedding
    torch.manual_seed(1)
    B, L, D = 16, 128, 256
    tabs = [torch.randn(V, D, device=gpu, requires_grad=True) for V in (5000, 512, 2)]
    ids = [torch.randint(0, 5000, (B, L), device=gpu), torch.arange(L, device=gpu).repeat(B, 1),
           torch.randint(0, 2, (B, L), device=gpu)]
    out = sum(embedding(i, t) for i, t in zip(ids, tabs))
    w = torch.randn_like(out)
    (out * w).sum().backward()
    for i, t in zip(ids, tabs):
        ref = torch.zeros_like(t, dtype=torch.float64).index_add_(0, i.reshape(-1), w.reshape(-1, D).double())
        assert torch.allclose(t.grad.double(), ref, rtol=1e-4, atol=1e-3)
