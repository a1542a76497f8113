"""Half-resolution residual of the dgrad epilogue (pw.hip BwdStats::resid_half): the compact data
gradient of a 1x1 stride-2 projection shortcut is added at the even positions of the block's conv1
dgrad instead of a zero-filled full-size tensor (zoo.ops.bn _HALF_RESID)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,H,W,Cin,K", [(2, 8, 6, 128, 256), (3, 14, 14, 256, 512),   # pw.hip
                                         (2, 6, 4, 96, 64)])                             # fallback (igemm)
def test_half_resid_equals_zero_interleaved(gpu, N, H, W, Cin, K):
    from zoo.ops import _kern
    torch.manual_seed(N + H + K)
    x = torch.randn(N, H, W, Cin, device=gpu).bfloat16()
    w = (torch.randn(K, Cin, device=gpu) * 0.05).bfloat16()
    r = torch.randn(N, H // 2, W // 2, K, device=gpu).bfloat16()
    full = torch.zeros(N, H, W, K, device=gpu, dtype=torch.bfloat16)
    full[:, ::2, ::2] = r
    a = _kern.conv_fwd(x, w, 1, 1, resid=r, resid_half=True)
    b = _kern.conv_fwd(x, w, 1, 1, resid=full)
    assert torch.equal(a, b)
    ref = (x.float().reshape(-1, Cin) @ w.float().t()).reshape(N, H, W, K) + full.float()
    assert ((a.float() - ref).norm() / ref.norm()).item() < 1e-2


def test_compact_shortcut_dgrad_matches_strided(gpu):
    from zoo.ops import _kern
    torch.manual_seed(1)
    dy = torch.randn(2, 7, 5, 64, device=gpu).bfloat16()
    w = (torch.randn(64, 32, device=gpu) * 0.1).bfloat16()
    full = _kern.conv_dgrad(dy, w, 64, 1, 1, 32, 14, 10, (2, 2), (0, 0))
    comp = _kern.conv_dgrad_s2_compact(dy, w, 64, 32)
    assert comp.shape == (2, 7, 5, 32)
    assert torch.allclose(full[:, ::2, ::2].float(), comp.float(), rtol=2e-2, atol=2e-2)
    assert not full[:, 1::2].any() and not full[:, :, 1::2].any()


def test_resnet50_half_resid_matches_full(gpu):
    """ResNet-50 training step with the compact shortcut gradient vs the zero-filled one. The fused
    step is not bitwise reproducible (atomic BN statistics), so the bar is the run-to-run spread of
    the zero-filled path itself: two runs of it, then the compact one against the first."""
    import zoo.models.image.resnet as R
    from zoo.ops import bn as B
    from zoo.ops import softmax_cross_entropy
    torch.manual_seed(0)
    m = R.resnet50(num_classes=100, zero_init_residual=True).to(gpu).train()
    x = torch.randn(16, 3, 96, 96, device=gpu)
    t = torch.randint(0, 100, (16,), device=gpu)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    grads, losses = [], []
    prev = B._HALF_RESID
    try:
        for half in (False, False, True):
            B._HALF_RESID = half
            m.load_state_dict(sd)
            m.zero_grad(set_to_none=True)
            loss = softmax_cross_entropy(m(x), t)
            loss.backward()
            losses.append(float(loss))
            grads.append([p.grad.detach().float().clone() for p in m.parameters()])
    finally:
        B._HALF_RESID = prev

    def worst(a, b):
        return min(F.cosine_similarity(u.flatten(), v.flatten(), dim=0).item()
                   for u, v in zip(a, b) if u.norm() > 0 and v.norm() > 0)
    noise = 1.0 - worst(grads[0], grads[1])
    diff = 1.0 - worst(grads[0], grads[2])
    print("loss %s, gradient 1-cos: run-to-run %.2e, compact vs full %.2e" % (losses, noise, diff))
    assert abs(losses[2] - losses[0]) <= 2 * abs(losses[1] - losses[0]) + 1e-3 * abs(losses[0])
    assert diff <= 3 * noise + 1e-3, (diff, noise)
