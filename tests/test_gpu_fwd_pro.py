"""Forward consumer-side BatchNorm apply (pw.hip EPI 1 prologue, conv_fwd pro_fwd): a 1x1 conv
consumes a conv -> BN -> ReLU unit's pre-BN output y and its affine, forms z = relu(A y + C) in
registers, writes z, and convolves it -- against a plain PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N,H,W,C,K,R", [(4, 14, 14, 64, 256, 1), (2, 28, 28, 128, 512, 1),
                                         (3, 9, 7, 64, 128, 1),
                                         (2, 8, 8, 256, 64, 1),     # K > 128: materialised fallback
                                         (2, 10, 10, 64, 64, 3)])   # 3x3 consumer: fallback
def test_conv_fwd_pro_fwd(gpu, N, H, W, C, K, R):
    from zoo.ops import _kern, native
    from zoo.ops.bn import stat_len
    torch.manual_seed(C + K + R)
    y = (torch.randn(N, H, W, C, device=gpu) * 1.5 + 0.3).bfloat16()
    gamma = torch.randn(C, device=gpu) * 0.7
    beta = torch.randn(C, device=gpu) * 0.2
    yf = y.float().reshape(-1, C)
    stats = torch.zeros(max(stat_len(C), 2 * C), device=gpu)
    stats[:C], stats[C:2 * C] = yf.sum(0), (yf * yf).sum(0)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    sm, si = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
    coef = native().bn_fwd_coef(stats, gamma, beta, rm, rv, sm, si, yf.shape[0], 1e-5, 0.1)
    mu, var = yf.mean(0), yf.var(0, unbiased=False)
    assert rel(sm, mu) < 1e-4 and rel(si, (var + 1e-5).rsqrt()) < 1e-4
    assert rel(rm, 0.1 * mu) < 1e-4 and rel(rv, 0.9 + 0.1 * yf.var(0, unbiased=True)) < 1e-4
    zref = F.relu((yf - mu) * (var + 1e-5).rsqrt() * gamma + beta).reshape(N, H, W, C)
    w = (torch.randn(K, R * R * C, device=gpu) * 0.05).bfloat16()
    z = torch.empty_like(y)
    st = torch.zeros(stat_len(K), device=gpu)
    out = _kern.conv_fwd(y, w, R, R, (1, 1), (R // 2, R // 2), stats=st, pro_fwd=(coef, z))
    assert rel(z, zref) < 1e-2
    ref = F.conv2d(zref.permute(0, 3, 1, 2), w.float().reshape(K, R, R, C).permute(0, 3, 1, 2),
                   padding=R // 2).permute(0, 2, 3, 1)
    assert rel(out, ref) < 1e-2
    # the conv's own output statistics still come out of its epilogue
    of = out.float().reshape(-1, K)
    assert rel(st[:K], of.sum(0)) < 2e-2


def test_resnet50_fwd_pro_matches_apply(gpu):
    """ResNet-50 training step with conv2's BN applied by conv3's prologue vs the separate apply
    pass: the bar is the run-to-run spread of the apply path itself (atomic statistics)."""
    import zoo.models.image.resnet as R
    from zoo.ops import softmax_cross_entropy
    torch.manual_seed(0)
    m = R.resnet50(num_classes=100, zero_init_residual=True).to(gpu).train()
    x = torch.randn(16, 3, 96, 96, device=gpu)
    t = torch.randint(0, 100, (16,), device=gpu)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    grads, losses, bufs = [], [], []
    prev = R.FWD_PRO
    try:
        for on in (False, False, True):
            R.FWD_PRO = on
            m.load_state_dict(sd)
            m.zero_grad(set_to_none=True)
            loss = softmax_cross_entropy(m(x), t)
            loss.backward()
            losses.append(float(loss))
            grads.append([p.grad.detach().float().clone() for p in m.parameters()])
            bufs.append([b.detach().float().clone() for b in m.buffers() if b.dtype.is_floating_point])
    finally:
        R.FWD_PRO = prev

    def worst(a, b):
        return min(F.cosine_similarity(u.flatten(), v.flatten(), dim=0).item()
                   for u, v in zip(a, b) if u.norm() > 0 and v.norm() > 0)
    noise = 1.0 - worst(grads[0], grads[1])
    diff = 1.0 - worst(grads[0], grads[2])
    print("loss %s, gradient 1-cos: run-to-run %.2e, prologue vs apply %.2e" % (losses, noise, diff))
    assert abs(losses[2] - losses[0]) <= 2 * abs(losses[1] - losses[0]) + 1e-3 * abs(losses[0])
    assert diff <= 3 * noise + 1e-3, (diff, noise)
    # running statistics updated the same way
    assert max(rel(b, a) for a, b in zip(bufs[0], bufs[2]) if a.norm() > 0) < 1e-2
