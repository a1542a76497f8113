"""BatchNorm backward of 1x1 conv -> BN units as the dgrad's prologue (csrc/kernels/bnfold.hip,
pw.hip PRO, zoo/ops/bn.py _BN_FOLD): the coefficient / apply kernels against fp32 PyTorch math,
the prologue dgrad against the dgrad of a materialised dy, and a bottleneck ResNet's gradients
with the prologue on vs the materialised BN backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _coef_ref(gamma, mean, inv, sums, M):
    K = gamma.numel()
    A = gamma * inv
    m1, m2 = sums[:K] / M, sums[K:2 * K] / M
    return A, -A * inv * m2, A * (mean * inv * m2 - m1)


def test_bnfold_coef_and_apply_match_fp32_formulas(gpu):
    from zoo.ops._native import native
    C_ = native()
    torch.manual_seed(0)
    K, M = 256, 1000
    gamma = torch.rand(K, device=gpu) + 0.5
    mean = torch.randn(K, device=gpu)
    inv = torch.rand(K, device=gpu) + 0.5
    sums = torch.zeros(2 * K + 64, device=gpu)
    sums[:2 * K] = torch.randn(2 * K, device=gpu) * 10
    dg0, db0 = torch.randn(K, device=gpu), torch.randn(K, device=gpu)
    dg, db = dg0.clone(), db0.clone()
    coef = C_.bnfold_coef(gamma, mean, inv, sums, M, dg, db)
    A, B, Cc = _coef_ref(gamma, mean, inv, sums, M)
    torch.testing.assert_close(coef, torch.cat([A, B, Cc]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dg, dg0 + sums[K:2 * K])
    torch.testing.assert_close(db, db0 + sums[:K])
    g = torch.randn(37, K, device=gpu).to(torch.bfloat16)
    y = torch.randn(37, K, device=gpu).to(torch.bfloat16)
    out = torch.empty_like(g)
    C_.bnpro_apply(g, y, coef, out)
    ref = A * g.float() + B * y.float() + Cc
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,K,N,det", [(4096, 64, 64, False), (3000, 64, 256, False), (4096, 256, 64, False),
                                       (2048, 128, 512, False), (512, 72, 128, False), (3000, 64, 256, True),
                                       (5000, 256, 256, False), (3000, 128, 128, False), (2000, 512, 64, False)])
def test_dgrad_prologue_matches_materialised_dy(gpu, M, K, N, det):
    """A 1x1 dgrad with the BN-backward prologue (pw.hip PRO at K = 64 / 128 / 256; K = 512, an odd
    width and the deterministic mode's partial statistics take the materialising fallback) against the same
    dgrad of dy materialised in fp32: the output, the written dy, with a residual operand and the
    producer's fused BN-backward epilogue."""
    from zoo.ops import _kern, deterministic, set_deterministic
    prev = deterministic()
    set_deterministic(det)
    try:
        _prologue_case(gpu, M, K, N)
    finally:
        set_deterministic(prev)


def _prologue_case(gpu, M, K, N):
    from zoo.ops import _kern
    torch.manual_seed(1)
    dev = gpu
    coef = torch.cat([torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1,
                      torch.randn(K, device=dev) * 0.1])
    g = torch.randn(M, K, device=dev).to(torch.bfloat16)
    y = torch.randn(M, K, device=dev).to(torch.bfloat16)
    wt = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)      # flipped 1x1 weight [N][K]
    resid = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dy_ref = (coef[:K] * g.float() + coef[K:2 * K] * y.float() + coef[2 * K:]).to(torch.bfloat16)
    x4 = lambda t: t.view(1, 1, M, t.shape[-1])
    # producer BN-backward epilogue operands (ReLU mask recomputed from its y with its affine)
    py = torch.randn(M, N, device=dev).to(torch.bfloat16)
    pm, pi = torch.randn(N, device=dev) * 0.1, torch.rand(N, device=dev) + 0.5
    pg, pb = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
    from zoo.ops.bn import stat_len
    s_ref = torch.zeros(stat_len(N), device=dev)
    s_pro = torch.zeros(stat_len(N), device=dev)
    ref = _kern.conv_fwd(x4(dy_ref), wt, 1, 1, resid=x4(resid), bstats=(None, x4(py), pm, pi, s_ref, pg, pb))
    dy_out = torch.empty_like(g)
    got = _kern.conv_fwd(x4(g), wt, 1, 1, resid=x4(resid), bstats=(None, x4(py), pm, pi, s_pro, pg, pb),
                         pro=(x4(y), coef, x4(dy_out)))
    torch.testing.assert_close(dy_out.float(), dy_ref.float(), rtol=1e-2, atol=1e-2)
    rel = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
    assert rel < 5e-3, rel
    srel = ((s_pro[:2 * N] - s_ref[:2 * N]).norm() / s_ref[:2 * N].norm()).item()
    assert srel < 5e-3, srel


def test_bnfold_matches_unfolded_backward(gpu):
    """A bottleneck ResNet (64-channel first stage: the prologue's units) with the 1x1 units' BN
    backward as the dgrad prologue vs materialised: the gradient difference is held to the
    run-to-run distance of the fp32-atomic reductions (as the BN-backward fusion test), overall
    and per weight / BN affine pair (+3 %), and the prologue really taken."""
    import zoo.models.image.resnet as R
    import zoo.ops.bn as B
    from zoo.ops import softmax_cross_entropy
    torch.manual_seed(0)
    m = R.ResNet(R.Bottleneck, [2, 1, 1, 1], num_classes=16, width=64).to(gpu)
    x = torch.randn(8, 3, 64, 64, device=gpu)
    y = torch.randint(0, 16, (8,), device=gpu)
    taken = [0]
    orig = B._fold_ok

    def spy(*a):
        ok = orig(*a)
        taken[0] += int(ok)
        return ok
    prev_fold = B._BN_FOLD[0]
    grads = []
    try:
        B._fold_ok = spy
        for mode in (False, False, True, True):
            B._BN_FOLD[0] = mode
            m.zero_grad(set_to_none=True)
            softmax_cross_entropy(m(x), y).backward()
            grads.append({n: p.grad.detach().double().clone() for n, p in m.named_parameters()})
    finally:
        B._BN_FOLD[0] = prev_fold
        B._fold_ok = orig
    # the first stage's two conv1 units (64 channels), both prologue runs
    assert taken[0] >= 2 * 2, taken

    def flat(gd):
        return torch.cat([v.flatten() for v in gd.values()])

    def dist(a, b):
        return ((a - b).norm() / b.norm()).item()
    u0, u1, f0, f1 = (flat(g) for g in grads)
    noise = max(dist(u0, u1), dist(f0, f1))
    err = (dist(f0, u0) + dist(f1, u1)) / 2
    assert err < 2.0 * noise + 0.005, (err, noise)
    # weights per tensor; BatchNorm affine gradients as each module's stacked [dgamma; dbeta] pair
    groups = {}
    for n in grads[0]:
        key = n.rsplit(".", 1)[0] + ".affine" if grads[0][n].dim() == 1 else n
        groups.setdefault(key, []).append(n)
    bad = {}
    for key, names in groups.items():
        u0g, u1g, f0g, f1g = (torch.cat([g[n].flatten() for n in names]) for g in grads)
        gnoise = max(dist(u0g, u1g), dist(f0g, f1g))
        gerr = dist(f0g, u0g)
        if gerr > 2.0 * gnoise + 0.03:
            bad[key] = (gerr, gnoise)
    assert not bad, bad
