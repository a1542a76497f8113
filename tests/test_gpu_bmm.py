"""Native batched GEMM (csrc/kernels/bmm.hip, zoo.ops.bmm) vs fp32 torch.matmul: every
transpose combination via strided views, batch broadcast, ragged sizes, fwd + bwd."""
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("shape_a,shape_b,ta,tb", [
    ((4, 37, 70), (4, 70, 51), False, False),
    ((4, 70, 37), (4, 70, 51), True, False),     # a given transposed
    ((4, 37, 70), (4, 51, 70), False, True),     # b given transposed
    ((3, 2, 64, 96), (1, 96, 128), False, False),  # broadcast batch
    ((8, 5, 33), (8, 33, 9), False, False),        # tiny / unaligned
])
def test_bmm_matches_fp32(shape_a, shape_b, ta, tb):
    from zoo.ops.bmm import bmm
    torch.manual_seed(0)
    dev = torch.device("cuda")
    a0 = torch.randn(*shape_a, device=dev)
    b0 = torch.randn(*shape_b, device=dev)
    a = (a0.transpose(-1, -2) if ta else a0).bfloat16().float().requires_grad_(True)
    b = (b0.transpose(-1, -2) if tb else b0).bfloat16().float().requires_grad_(True)
    ref = torch.matmul(a, b)
    out = bmm(a, b)
    assert out.shape == ref.shape
    assert ((out - ref).norm() / ref.norm()).item() < 1e-2
    g = torch.randn_like(ref)
    ga, gb = torch.autograd.grad(ref, (a, b), g)
    na, nb = torch.autograd.grad(out, (a, b), g)
    assert ((na - ga).norm() / ga.norm()).item() < 1e-2
    assert ((nb - gb).norm() / gb.norm()).item() < 1e-2


@pytest.mark.gpu
def test_autograd_batch_dot_runs_native():
    from zoo.pipeline.api import autograd as A
    torch.manual_seed(1)
    x = torch.randn(6, 10, 16, device="cuda")
    y = torch.randn(6, 12, 16, device="cuda")
    out = A.batch_dot(x, y, axes=(2, 2))
    ref = torch.matmul(x, y.transpose(1, 2))
    assert ((out - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.gpu
def test_convlstm2d_native_matches_cpu_reference():
    """ConvLSTM2D on the GPU (input + recurrent convs on the native MFMA conv) vs the
    fp32 CPU implementation of the same layer, forward and parameter gradients."""
    import copy
    from zoo.pipeline.api.keras.layers import ConvLSTM2D
    torch.manual_seed(3)
    lay = ConvLSTM2D(6, 3, 3, return_sequences=True, inner_activation="sigmoid", input_shape=(4, 3, 8, 8))
    lay._ensure_built((None, 4, 3, 8, 8))
    x = torch.randn(2, 4, 3, 8, 8)
    ref_l = copy.deepcopy(lay)
    ref = ref_l(x)
    ref.sum().backward()
    gl = lay.cuda()
    out = gl(x.cuda())
    assert out.shape == ref.shape
    assert ((out.float().cpu() - ref).norm() / ref.norm()).item() < 3e-2
    out.float().sum().backward()
    for name in ("Wx", "Wh", "b"):
        a, r = getattr(gl, name).grad.float().cpu(), getattr(ref_l, name).grad
        assert ((a - r).norm() / r.norm()).item() < 5e-2, name


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("axis", [-1, 1])
def test_native_reduce_matches_torch(op, axis):
    from zoo.ops.reduce import reduce
    torch.manual_seed(4)
    x = torch.randn(6, 37, 130, device="cuda", requires_grad=True)
    ref_fn = {"sum": lambda t: t.sum(axis), "mean": lambda t: t.mean(axis),
              "max": lambda t: t.amax(axis), "min": lambda t: t.amin(axis)}[op]
    ref = ref_fn(x)
    out = reduce(x, axis, op)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-5)
    g = torch.randn_like(ref)
    (gr,) = torch.autograd.grad(ref, x, g)
    (gn,) = torch.autograd.grad(out, x, g)
    assert torch.allclose(gn, gr, atol=1e-5)


@pytest.mark.gpu
def test_native_l2_normalize_fwd_bwd():
    from zoo.ops.reduce import l2_normalize
    from zoo.pipeline.api import autograd as A
    torch.manual_seed(5)
    x = torch.randn(8, 20, 300, device="cuda", requires_grad=True)
    for axis in (-1, 1):
        ref = x / torch.sqrt(torch.clamp((x * x).sum(dim=axis, keepdim=True), min=1e-12))
        out = l2_normalize(x, axis)
        assert torch.allclose(out, ref, atol=1e-5)
        g = torch.randn_like(ref)
        (gr,) = torch.autograd.grad(ref, x, g)
        (gn,) = torch.autograd.grad(out, x, g)
        assert torch.allclose(gn, gr, atol=1e-4)
    assert torch.allclose(A.sum(x, axis=2), x.sum(2), atol=1e-4)


@pytest.mark.gpu
def test_ssd_native_matching_matches_reference():
    """MultiBoxLoss matching on the native kernel vs the per-image torch matcher."""
    from zoo.models.image.objectdetection.ssd import MultiBoxLoss, SSDConfig, prior_boxes
    torch.manual_seed(6)
    priors = prior_boxes(SSDConfig()).float()
    crit = MultiBoxLoss(num_classes=21)
    targets = []
    for n in (3, 0, 7, 1):
        xy = torch.rand(n, 2) * 0.7
        wh = torch.rand(n, 2) * 0.3 + 0.02
        lab = torch.randint(1, 21, (n, 1)).float()
        targets.append(torch.cat([lab, xy, xy + wh], 1))
    ref_l, ref_c = [], []
    for t in targets:
        l, c = crit.match(t[:, 1:], t[:, 0], priors)
        ref_l.append(l)
        ref_c.append(c)
    ref_l, ref_c = torch.stack(ref_l), torch.stack(ref_c)
    loc_t, conf_t = crit.match_native([t.cuda() for t in targets], priors.cuda())
    assert torch.equal(conf_t.cpu(), ref_c)
    pos = ref_c != 0
    assert torch.allclose(loc_t.cpu()[pos], ref_l[pos], atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("P,frac", [(8732, 0.02), (8732, 0.4), (3000, 0.0), (1500, 0.9)])
def test_ssd_native_mining_matches_stable_rank(P, frac):
    """Hard negative mining kernel (radix select, detect.hip ssd_mine) vs the stable-sort rank on
    the CPU: identical masks, including ties (quantised losses) and the P - 1 clamp."""
    from zoo.models.image.objectdetection.ssd import mine_hard_negatives
    torch.manual_seed(7)
    B = 5
    ce = torch.rand(B, P)
    ce[1] = (ce[1] * 8).floor() / 8                 # heavy ties
    ce[2, : P // 3] = 0.0
    pos = torch.rand(B, P) < frac
    pos[3] = False                                    # no positives: nothing mined
    ref = mine_hard_negatives(ce, pos, 3.0)
    out = mine_hard_negatives(ce.cuda(), pos.cuda(), 3.0).cpu()
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 38, 38, 512), (3, 5, 7, 64), (2, 1, 1, 1024)])
def test_normalize_scale_native_fwd_bwd(shape):
    """SSD conv4_3 NormalizeScale on the fused kernels vs the fp32 torch composition."""
    from zoo.models.image.objectdetection.ssd import NormalizeScale
    torch.manual_seed(8)
    m = NormalizeScale(shape[-1]).cuda()
    with torch.no_grad():
        m.weight.uniform_(5, 25)
    x = torch.relu(torch.randn(*shape, device="cuda")).bfloat16()
    xr = x.float().requires_grad_(True)
    wr = m.weight.detach().clone().requires_grad_(True)
    ref = xr / (xr.pow(2).sum(-1, keepdim=True).sqrt() + m.eps) * wr
    xn = x.clone().requires_grad_(True)
    out = m(xn)
    assert out.dtype == torch.bfloat16
    assert ((out.float() - ref).norm() / ref.norm()).item() < 1e-2
    g = torch.randn_like(ref).bfloat16()
    gx, gw = torch.autograd.grad(ref, (xr, wr), g.float())
    nx, nw = torch.autograd.grad(out, (xn, m.weight), g)
    assert ((nx.float() - gx).norm() / gx.norm()).item() < 2e-2
    assert ((nw - gw).norm() / gw.norm()).item() < 1e-2
