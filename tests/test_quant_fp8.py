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
