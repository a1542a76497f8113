"""Static-int8 implicit-GEMM conv (csrc/kernels/qconv.hip) against its float64 model
(zoo.ops.qresnet.qconv_ref), and the calibrated int8 ResNet against the bf16 model."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [(2, 14, 64, 64, 1, 1, 0), (2, 14, 64, 128, 3, 1, 1),
                                                  (3, 15, 32, 64, 3, 2, 1), (2, 16, 128, 256, 1, 2, 0),
                                                  (1, 7, 512, 2048, 1, 1, 0), (4, 28, 16, 72, 3, 1, 1)])
@pytest.mark.parametrize("resid,relu,out_bf16", [(False, True, False), (True, True, False), (True, False, True)])
def test_qconv_matches_float64_model(gpu, N, H, C, K, R, stride, pad, resid, relu, out_bf16):
    from zoo.ops.qresnet import qconv, qconv_ref
    g = torch.Generator().manual_seed(N * 1000 + C + K)
    xq = torch.randint(-127, 128, (N, H, H, C), generator=g, dtype=torch.int8)
    wq = torch.randint(-127, 128, (K, R * R * C), generator=g, dtype=torch.int8)
    cs = (torch.rand(K, generator=g) * 2e-4 + 1e-5).float()
    b = (torch.randn(K, generator=g) * 3).float()
    P = (H + 2 * pad - R) // stride + 1
    rq = torch.randint(-127, 128, (N, P, P, K), generator=g, dtype=torch.int8) if resid else None
    ref = qconv_ref(xq, wq, R, R, stride, pad, cs, b, rq, 0.37, relu, out_bf16)
    out = qconv(xq.to(gpu), wq.to(gpu), R, R, stride, pad, cs.to(gpu), b.to(gpu),
                None if rq is None else rq.to(gpu), 0.37, relu, out_bf16).cpu()
    assert out.shape == ref.shape and out.dtype == ref.dtype
    if out_bf16:
        assert torch.allclose(out.float(), ref.float(), rtol=1e-2, atol=1e-2)
    else:
        d = (out.int() - ref.int()).abs()
        assert int(d.max()) <= 1 and float((d > 0).float().mean()) < 1e-3   # fp32 vs fp64 rounding ties


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [(2, 14, 64, 128, 3, 1, 1), (3, 15, 32, 64, 3, 2, 1),
                                                  (2, 14, 64, 64, 1, 1, 0), (2, 16, 128, 256, 1, 2, 0)])
@pytest.mark.parametrize("qflags,resid,relu,out_bf16", [(7, True, True, False), (3, False, True, False),
                                                        (1, False, True, True), (5, True, False, True),
                                                        (1, True, False, False)])
def test_qconv_unsigned_code_matches_float64_model(gpu, N, H, C, K, R, stride, pad, qflags, resid, relu, out_bf16):
    """Offset-coded unsigned int8 operands (QF_IN_U8 input incl. its padding taps, QF_OUT_U8
    output, QF_RES_U8 residual) against the float64 model."""
    from zoo.ops.qresnet import qconv, qconv_ref
    g = torch.Generator().manual_seed(N * 1000 + C + K + qflags)
    xq = torch.randint(-128, 128, (N, H, H, C), generator=g, dtype=torch.int8)
    wq = torch.randint(-127, 128, (K, R * R * C), generator=g, dtype=torch.int8)
    cs = (torch.rand(K, generator=g) * 2e-4 + 1e-5).float()
    b = (torch.randn(K, generator=g) * 3).float()
    P = (H + 2 * pad - R) // stride + 1
    rq = torch.randint(-128, 128, (N, P, P, K), generator=g, dtype=torch.int8) if resid else None
    ref = qconv_ref(xq, wq, R, R, stride, pad, cs, b, rq, 0.37, relu, out_bf16, qflags=qflags)
    out = qconv(xq.to(gpu), wq.to(gpu), R, R, stride, pad, cs.to(gpu), b.to(gpu),
                None if rq is None else rq.to(gpu), 0.37, relu, out_bf16, qflags=qflags).cpu()
    assert out.shape == ref.shape and out.dtype == ref.dtype
    if out_bf16:
        assert torch.allclose(out.float(), ref.float(), rtol=1e-2, atol=1e-2)
    else:
        d = (out.int() - ref.int()).abs()
        assert int(d.max()) <= 1 and float((d > 0).float().mean()) < 1e-3


def test_unsigned_quantize_and_gap(gpu):
    from zoo import ops
    from zoo.ops.qresnet import _dequant, quantize_act
    torch.manual_seed(3)
    x = (torch.rand(2, 5, 7, 32, device=gpu) * 3).bfloat16()
    s = (x.float().reshape(-1, 32).amax(0) / 255).clamp_min(1e-6)
    q = quantize_act(x, s, "int8", u8=True)
    qc = quantize_act(x.cpu(), s.cpu(), "int8", u8=True)
    d = (q.cpu().int() - qc.int()).abs()      # fp32 x * (1/s) on the GPU vs float64 x / s: rounding ties
    assert int(d.max()) <= 1 and float((d > 0).float().mean()) < 1e-2
    assert int(q.min()) >= -128 and ((_dequant(q, s, True) - x.float()).abs() <= s / 2 + 1e-3).all()
    feat = ops.native().gap_i8(q, 1.0, s.float().contiguous(), True)
    ref = _dequant(q, s, True).mean((1, 2))
    assert torch.allclose(feat.float(), ref, rtol=1e-2, atol=1e-3)


@pytest.fixture(scope="module")
def trained_resnet50(gpu):
    """ResNet-50 fitted to a learnable synthetic task (zoo.utils.synthetic): quantization is judged
    on confident, input-dependent predictions -- a random-init net's logits barely depend on the
    input, so its top-1 flips on noise far below any real model's margins."""
    from zoo.models.image.resnet import resnet50
    from zoo.utils.synthetic import class_templates, train_briefly
    torch.manual_seed(0)
    m = resnet50(num_classes=16).to(gpu)
    T = class_templates(16, 128, device=gpu)
    acc = train_briefly(m, T)
    assert acc > 0.9, acc
    return m, T


def _quant_agreement(trained, fmt, act_scales=None):
    from zoo.ops.qresnet import Fp8ResNet, Int8ResNet
    from zoo.utils.synthetic import agreement, sample
    m, T = trained
    calib, _ = sample(T, 64, seed=11)
    x, _ = sample(T, 128, seed=12)
    with torch.no_grad():
        ref = m(x).float()
    q = (Fp8ResNet if fmt == "fp8" else Int8ResNet)(m, calib, act_scales=act_scales)
    with torch.no_grad():
        out = q(x).float()
    assert out.shape == ref.shape and torch.isfinite(out).all()
    return agreement(out, ref)


def test_int8_resnet_tracks_bf16_model(gpu, trained_resnet50):
    """Per-sample agreement with the bf16 model: top-1 and the cosine of each sample's
    mean-centred logits (not a flattened cosine, which the shared logit offset dominates)."""
    top1, cos = _quant_agreement(trained_resnet50, "int8")
    assert top1 >= 0.9 and cos >= 0.9, (top1, cos)


def test_int8_signed_code_tracks_bf16_model(gpu, trained_resnet50):
    """The symmetric (signed) activation code, act_u8=False, still tracks the model."""
    from zoo.ops.qresnet import Int8ResNet
    from zoo.utils.synthetic import agreement, sample
    m, T = trained_resnet50
    calib, _ = sample(T, 64, seed=11)
    x, _ = sample(T, 128, seed=12)
    with torch.no_grad():
        ref = m(x).float()
        top1, cos = agreement(Int8ResNet(m, calib, act_u8=False)(x).float(), ref)
    assert top1 >= 0.9 and cos >= 0.9, (top1, cos)


def test_int8_mse_scales_track_bf16_model(gpu, trained_resnet50):
    """MSE-searched per-channel activation clipping: scales never exceed the channel absmax, and
    the twin tracks the bf16 model as well as the absmax-calibrated one."""
    top1, cos = _quant_agreement(trained_resnet50, "int8", act_scales="mse")
    assert top1 >= 0.9 and cos >= 0.9, (top1, cos)


def test_int8_mixed_precision_blocks(gpu, trained_resnet50):
    """Per-block bf16 fallback: the calibrated per-block error is reported for every residual
    block, chosen blocks run on the bf16 kernels between dequantise / requantise boundaries, and
    with every block in bf16 the twin reproduces the bf16 model (only the stem / classifier path
    is shared)."""
    from zoo.ops.qresnet import Int8ResNet
    from zoo.utils.synthetic import agreement, sample
    m, T = trained_resnet50
    calib, _ = sample(T, 64, seed=11)
    x, _ = sample(T, 128, seed=12)
    with torch.no_grad():
        ref = m(x).float()
    q = Int8ResNet(m, calib, bf16_blocks=(0, 7, 15))
    assert len(q.block_err) == 16 and all(0 < e < 0.5 for e in q.block_err), q.block_err
    with torch.no_grad():
        top1, cos = agreement(q(x).float(), ref)
    assert top1 >= 0.9 and cos >= 0.9, (top1, cos)
    qa = Int8ResNet(m, calib, max_block_err=0.0)          # every block above 0 -> all bf16
    assert qa.bf16_blocks == set(range(16))
    with torch.no_grad():
        out = qa(x).float()
    assert ((out - ref).norm() / ref.norm()).item() < 1e-2


def test_inference_model_static_int8_with_hipgraph(gpu):
    """InferenceModel.load_module(blas=False, calib_data=...) serves the calibrated int8
    twin through the hipGraph replica path; predictions track the bf16 model."""
    import numpy as np
    from zoo.models.image.resnet import resnet18
    from zoo.pipeline.inference import InferenceModel
    torch.manual_seed(1)
    m = resnet18(num_classes=10).to(gpu).eval()
    x = torch.randn(8, 3, 64, 64)
    with torch.no_grad():
        ref = m(x.to(gpu)).float().cpu().numpy()
    im = InferenceModel(2, device=gpu).load_module(m, blas=False, calib_data=torch.randn(8, 3, 64, 64))
    from zoo.ops.qresnet import Int8ResNet
    assert isinstance(im.model, Int8ResNet)
    out = im.predict(x)
    out2 = im.predict(x)       # graph replay
    assert np.allclose(out, out2)
    cos = float((out * ref).sum() / (np.linalg.norm(out) * np.linalg.norm(ref)))
    assert cos > 0.95, cos


# ---- OCP fp8 (e4m3fn) twin: v_mfma_f32_16x16x128_f8f6f4 ----
@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [(2, 14, 64, 64, 1, 1, 0), (2, 14, 64, 128, 3, 1, 1),
                                                  (3, 15, 32, 64, 3, 2, 1), (1, 7, 512, 2048, 1, 1, 0),
                                                  (4, 28, 16, 72, 3, 1, 1)])
@pytest.mark.parametrize("resid,relu,out_bf16", [(False, True, False), (True, True, False), (True, False, True)])
def test_fp8conv_matches_float64_model(gpu, N, H, C, K, R, stride, pad, resid, relu, out_bf16):
    from zoo.ops.qresnet import qconv, qconv_ref, to_fp8
    g = torch.Generator().manual_seed(N * 1000 + C + K)
    xq = to_fp8(torch.randn(N, H, H, C, generator=g) * 40)
    wq = to_fp8(torch.randn(K, R * R * C, generator=g) * 40)
    cs = (torch.rand(K, generator=g) * 2e-4 + 1e-5).float()
    b = (torch.randn(K, generator=g) * 3).float()
    P = (H + 2 * pad - R) // stride + 1
    rq = to_fp8(torch.randn(N, P, P, K, generator=g) * 40) if resid else None
    ref = qconv_ref(xq, wq, R, R, stride, pad, cs, b, rq, 0.37, relu, out_bf16)
    out = qconv(xq.to(gpu), wq.to(gpu), R, R, stride, pad, cs.to(gpu), b.to(gpu),
                None if rq is None else rq.to(gpu), 0.37, relu, out_bf16).cpu()
    assert out.shape == ref.shape and out.dtype == ref.dtype
    o, r = out.float(), ref.float()
    if out_bf16:
        assert torch.allclose(o, r, rtol=1e-2, atol=1e-2)
    else:
        # fp32 vs fp64 accumulation can move a value across an e4m3 rounding boundary (one ulp,
        # 2^-3 relative) on rare ties
        bad = (o - r).abs() > 0.13 * r.abs() + 1e-6
        assert float(bad.float().mean()) < 1e-3 and float(((o != r).float()).mean()) < 2e-2


def test_fp8_resnet_tracks_bf16_model(gpu, trained_resnet50):
    top1, cos = _quant_agreement(trained_resnet50, "fp8")
    assert top1 >= 0.9 and cos >= 0.9, (top1, cos)


def test_inference_model_fp8(gpu):
    import numpy as np
    from zoo.models.image.resnet import resnet18
    from zoo.ops.qresnet import Fp8ResNet
    from zoo.pipeline.inference import InferenceModel
    torch.manual_seed(1)
    m = resnet18(num_classes=10).to(gpu).eval()
    x = torch.randn(8, 3, 64, 64)
    with torch.no_grad():
        ref = m(x.to(gpu)).float().cpu().numpy()
    im = InferenceModel(1, device=gpu).load_module(m, blas=False, calib_data=torch.randn(8, 3, 64, 64),
                                                   qdtype="fp8")
    assert isinstance(im.model, Fp8ResNet)
    out = im.predict(x)
    cos = float((out * ref).sum() / (np.linalg.norm(out) * np.linalg.norm(ref)))
    assert cos > 0.9, cos
