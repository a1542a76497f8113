"""int8 quantized inference (zoo.ops.quant; BigDL quantize() parity, HK23).

CPU: the float64 integer reference path vs plain fp32 layers. GPU: the int8
MFMA kernels (csrc/kernels/quant.hip) vs that reference, bit-for-bit on the
integer accumulation (compared after the fp32 rescale)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from zoo.ops import quant as Q


def test_quantize_weight_roundtrip():
    torch.manual_seed(0)
    w = torch.randn(10, 37)
    q, s = Q.quantize_weight(w)
    assert q.shape == (10, 48) and q.dtype == torch.int8 and (q[:, 37:] == 0).all()
    rec = q[:, :37].float() * s[:, None]
    assert (rec - w).abs().max() <= s.max() / 2 + 1e-6


def test_qconv_reference_close_to_float_conv():
    torch.manual_seed(1)
    x = torch.randn(2, 9, 9, 8)
    w4 = torch.randn(16, 3, 3, 8) * 0.1
    qw, s = Q.quantize_weight(w4.reshape(16, -1))
    y = Q.qconv_nhwc(x, qw, s, None, (3, 3), (2, 2), (1, 1))
    ref = F.conv2d(x.permute(0, 3, 1, 2), w4.permute(0, 3, 1, 2), stride=2, padding=1).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert (y - ref).norm() / ref.norm() < 0.02


def test_quantize_small_resnet_cpu():
    from zoo.models.image.resnet import BasicBlock, ResNet
    torch.manual_seed(2)
    m = ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=16).eval()
    for mod in m.modules():  # non-trivial BN statistics to fold
        if hasattr(mod, "running_var"):
            mod.running_var.uniform_(0.5, 2.0)
            mod.running_mean.uniform_(-0.2, 0.2)
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        ref = m(x).float()
        Q.quantize(m)
        out = m(x).float()
    assert Q.is_quantized(m)
    assert (out - ref).norm() / ref.norm() < 0.1


def test_quantized_keras_dense_and_torch_linear():
    from zoo.pipeline.api.keras.layers import Dense
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(3)
    km = Sequential()
    km.add(Dense(16, activation="relu", input_shape=(12,)))
    km.add(Dense(4))
    x = torch.randn(5, 12)
    with torch.no_grad():
        ref = km(x)
        Q.quantize(km)
        out = km(x)
    assert (out - ref).norm() / ref.norm() < 0.05
    tm = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(), torch.nn.Flatten(),
                             torch.nn.Linear(8 * 6 * 6, 5))
    xi = torch.randn(2, 3, 6, 6)
    with torch.no_grad():
        r = tm(xi)
        Q.quantize(tm)
        o = tm(xi)
    assert isinstance(tm[0], Q.QuantizedConv2d) and isinstance(tm[3], Q.QuantizedLinear)
    assert (o - r).norm() / r.norm() < 0.05


def test_inference_model_blas_false_quantizes():
    from zoo.pipeline.inference import InferenceModel
    torch.manual_seed(4)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    im = InferenceModel(device="cpu").load_module(net, blas=False)
    assert Q.is_quantized(im.model)
    out = im.predict(np.random.randn(4, 8).astype(np.float32))
    assert np.asarray(out).shape == (4, 3)


@pytest.mark.gpu
def test_int8_kernels_match_reference():
    from zoo.ops._native import native
    assert hasattr(native(), "qgemm"), "int8 kernels not built"
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    for (n, h, w, c, k, r, st, pd) in [(2, 14, 14, 64, 96, 3, 1, 1), (3, 9, 11, 24, 40, 1, 2, 0),
                                        (1, 7, 7, 200, 130, 3, 2, 1)]:
        x = torch.randn(n, h, w, c)
        w4 = torch.randn(k, r, r, c) * 0.05
        qw, s = Q.quantize_weight(w4.reshape(k, -1))
        bias = torch.randn(k)
        P = (h + 2 * pd - r) // st + 1
        Qd = (w + 2 * pd - r) // st + 1
        resid = torch.randn(n, P, Qd, k).to(torch.bfloat16)
        ref = Q.qconv_nhwc(x, qw, s, bias, (r, r), (st, st), (pd, pd), resid=resid.float(), relu=True)
        got = Q.qconv_nhwc(x.to(dev), qw.to(dev), s.to(dev), bias.to(dev), (r, r), (st, st), (pd, pd),
                           resid=resid.to(dev), relu=True, out_f32=True).cpu()
        assert torch.allclose(got, ref, rtol=1e-4, atol=1e-3), (got - ref).abs().max()


@pytest.mark.gpu
def test_int8_resnet50_agrees_with_bf16():
    from zoo.models.image.resnet import resnet50
    dev = torch.device("cuda:0")
    torch.manual_seed(6)
    m = resnet50(num_classes=1000).to(dev).eval()
    x = torch.randn(8, 3, 224, 224, device=dev)
    with torch.no_grad():
        ref = m(x).float()
        Q.quantize(m)
        out = m(x).float()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 0.15, rel
    cos = F.cosine_similarity(out.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.98, cos
