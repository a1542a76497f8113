"""CPU side of the fp8 (OCP e4m3fn) static-quantized ResNet: the float64 kernel model and the
calibrated twin run on the CPU and track the fp32 model (the GPU kernel is checked against the
same model in test_gpu_qconv.py)."""
import torch


def test_fp8_reference_conv_matches_dequantized_float_conv():
    import torch.nn.functional as F
    from zoo.ops.qresnet import qconv_ref, to_fp8
    g = torch.Generator().manual_seed(0)
    xq = to_fp8(torch.randn(2, 9, 9, 16, generator=g) * 30)
    wq = to_fp8(torch.randn(32, 9 * 16, generator=g) * 30)
    cs = torch.full((32,), 1e-3)
    out = qconv_ref(xq, wq, 3, 3, 1, 1, cs, None, out_bf16=True).float()
    ref = F.conv2d(xq.float().permute(0, 3, 1, 2), wq.float().reshape(32, 3, 3, 16).permute(0, 3, 1, 2),
                   padding=1).permute(0, 2, 3, 1) * 1e-3
    assert torch.allclose(out, ref, rtol=1e-2, atol=1e-2)
    q = qconv_ref(xq, wq, 3, 3, 1, 1, cs, None)
    assert q.dtype == torch.float8_e4m3fn


def test_fp8_resnet_cpu_tracks_fp32():
    from zoo.models.image.resnet import resnet18
    from zoo.ops.quant import quantize
    from zoo.ops.qresnet import Fp8ResNet
    torch.manual_seed(0)
    m = resnet18(num_classes=10).eval()
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        ref = m(x).float()
        q = quantize(m, torch.randn(4, 3, 64, 64), dtype="fp8")
        assert isinstance(q, Fp8ResNet)
        out = q(x).float()
    cos = torch.nn.functional.cosine_similarity(out.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.9, cos


def test_fp8_needs_calibrated_resnet():
    import pytest
    from zoo.ops.quant import quantize
    with pytest.raises(ValueError):
        quantize(torch.nn.Sequential(torch.nn.Linear(4, 4)), dtype="fp8")


def test_unsigned_int8_code_reference_matches_float_conv():
    """Offset-coded unsigned activations (qresnet QF_IN_U8): q = round(x / s) - 128, padding taps
    at the code of 0, and the 128 * sum(w) term folded into the bias reproduce the float conv of the
    dequantised input (CPU float64 model of qconv.hip)."""
    import torch.nn.functional as F
    from zoo.ops.qresnet import QF_IN_U8, QF_OUT_U8, _dequant, _sat_u8, qconv_ref
    torch.manual_seed(4)
    x = torch.rand(2, 9, 9, 16) * 5
    s = 5.0 / 255
    xq = _sat_u8(x.double() / s).to(torch.int8)
    wq = torch.randint(-127, 128, (8, 3 * 3 * 16), dtype=torch.int8)
    cs = torch.full((8,), 1e-3)
    b = torch.randn(8)
    bias = b + cs * 128.0 * wq.float().sum(1)
    out = qconv_ref(xq, wq, 3, 3, 1, 1, cs, bias, out_bf16=True, qflags=QF_IN_U8).double()
    xd = _dequant(xq, s, True).double() / s
    w4 = wq.double().reshape(8, 3, 3, 16).permute(0, 3, 1, 2)
    ref = F.conv2d(xd.permute(0, 3, 1, 2), w4, padding=1).permute(0, 2, 3, 1) * cs.double() + b.double()
    assert ((out - ref).norm() / ref.norm()).item() < 1e-2
    # unsigned output: the code of relu(v), 255 levels
    o8 = qconv_ref(xq, wq, 3, 3, 1, 1, cs, bias, relu=True, qflags=QF_IN_U8 | QF_OUT_U8)
    assert o8.dtype == torch.int8
    assert torch.equal(o8, (torch.clamp(torch.round(ref.clamp_min(0)), 0, 255) - 128).to(torch.int8))
