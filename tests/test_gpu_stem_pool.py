"""Fused stem BatchNorm -> ReLU -> max-pool (csrc/kernels/bn.hip bn_relu_maxpool_*) against a
plain PyTorch fp32 reference of the same composition (forward, running statistics, and the
gradients of the raw input, gamma and beta), plus the ResNet-50 wiring."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N,H,W,C,k,s,p", [(2, 112, 112, 64, 3, 2, 1), (3, 15, 17, 128, 3, 2, 1),
                                           (2, 9, 8, 16, 3, 2, 1),      # compile-time stem geometry
                                           (2, 10, 12, 16, 3, 2, 1), (1, 8, 6, 256, 3, 2, 1), (1, 8, 8, 256, 3, 2, 1),   # fwd2 pairs
                                           (2, 10, 13, 32, 2, 2, 0), (2, 11, 9, 64, 3, 1, 1)])  # generic
def test_bn_relu_maxpool_vs_fp32(gpu, N, H, W, C, k, s, p):
    from zoo.ops.bn import ShortcutBN, bn_relu_maxpool, stat_len
    torch.manual_seed(0)
    y = (torch.randn(N, H, W, C, device=gpu) * 2 + 0.5).bfloat16()
    gamma = (torch.randn(C, device=gpu) * 0.8).requires_grad_(True)   # mixed signs: min-pool channels
    beta = (torch.randn(C, device=gpu) * 0.3).requires_grad_(True)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    holder = ShortcutBN(rm, rv)
    yf = y.float().reshape(-1, C)
    st = torch.zeros(stat_len(C), device=gpu)
    st[:C], st[C:2 * C] = yf.sum(0), (yf * yf).sum(0)
    holder.stats = st
    yg = y.clone().requires_grad_(True)
    out = bn_relu_maxpool(yg, holder, gamma, beta, 1e-5, 0.1, (k, k), (s, s), (p, p))

    yr = y.float().permute(0, 3, 1, 2).requires_grad_(True)
    gr, br = gamma.detach().clone().requires_grad_(True), beta.detach().clone().requires_grad_(True)
    rm2, rv2 = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    zr = F.relu(F.batch_norm(yr, rm2, rv2, gr, br, training=True, momentum=0.1, eps=1e-5))
    outr = F.max_pool2d(zr, k, s, p)
    assert out.shape == (N, outr.shape[2], outr.shape[3], C)
    assert rel(out, outr.permute(0, 2, 3, 1)) < 1e-2
    assert rel(rm, rm2) < 1e-4 and rel(rv, rv2) < 1e-4
    dout = torch.randn_like(out)
    out.backward(dout)
    outr.backward(dout.float().permute(0, 3, 1, 2))
    assert rel(yg.grad, yr.grad.permute(0, 2, 3, 1)) < 3e-2
    assert rel(gamma.grad, gr.grad) < 2e-2
    assert rel(beta.grad, br.grad) < 2e-2


def test_resnet50_stem_fusion_matches_unfused(gpu):
    """ResNet-50 training forward/backward with the stem fusion on vs off: same loss and
    matching stem-weight / stem-BN gradients (the only difference is bf16 rounding of the
    materialised stem BN output in the unfused path). Zero-initialised residual gammas, as
    in test_gpu_resnet50_parity: with gamma=1 the stem gradient at init is dominated by bf16
    noise accumulated over 50 layers (torch autocast itself lands at cosine 0.1-0.3)."""
    import zoo.models.image.resnet as R
    from zoo.ops import softmax_cross_entropy
    torch.manual_seed(0)
    m = R.resnet50(num_classes=1000, zero_init_residual=True).to(gpu).train()
    x = torch.randn(8, 3, 224, 224, device=gpu)
    t = torch.randint(0, 1000, (8,), device=gpu)
    grads, losses = [], []
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for fuse in (False, True):
        m.load_state_dict(sd)
        m.zero_grad(set_to_none=True)
        R.FUSE_STEM_POOL = fuse
        try:
            loss = softmax_cross_entropy(m(x), t)
            loss.backward()
        finally:
            R.FUSE_STEM_POOL = True
        losses.append(float(loss))
        grads.append([p.grad.detach().float().clone() for p in (m.stem.weight, m.stem.gamma, m.stem.beta)])
    assert abs(losses[0] - losses[1]) < 2e-2 * abs(losses[0])
    cs = [F.cosine_similarity(a.flatten(), b.flatten(), dim=0).item() for a, b in zip(*grads)]
    print("stem fusion on/off: loss %s grad cosines %s" % (losses, cs))
    for a, b in zip(*grads):
        assert F.cosine_similarity(a.flatten(), b.flatten(), dim=0).item() > 0.98
