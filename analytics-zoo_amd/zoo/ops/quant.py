"""int8 quantized inference (BigDL ``quantize()``: InferenceModelFactory.scala:33,47,
ImageModel.scala:133-145).

Scheme: symmetric int8 weights with one scale per output channel, activations
quantized on the fly with one dynamic per-tensor scale (absmax / 127), int32
accumulation on the int8 matrix cores, fp32 rescale + bias (+ residual) (+ ReLU)
in the GEMM epilogue (csrc/kernels/quant.hip). Convolutions run as an int8
im2col (NHWC, packed-weight k order) followed by the same GEMM.

``quantize(model)`` converts, in place, every supported layer of an eval-mode
model: ResNet ConvBN units (BatchNorm folded into the int8 weights), the ResNet
classifier, zoo Keras ``Dense`` layers and ``torch.nn.Linear`` / ``Conv2d``.
On the CPU the same integer arithmetic runs exactly in float64 (the reference
path the GPU kernels are tested against).

This module is the DYNAMIC path (no calibration data: per-call activation absmax, im2col +
GEMM; any model). With calibration data a zoo ResNet takes the STATIC path instead --
``quantize(model, calib_data)`` returns a :class:`zoo.ops.qresnet.Int8ResNet`, whose
convolutions are one implicit-GEMM int8 kernel each with the whole unit fused in the
epilogue (tools/quant_bench.py, MI355X, ResNet-50 b256: static int8 60.2k img/s vs bf16
41.1k vs this dynamic path 11.1k; profiles/resnet50_infer_int8_r2.md).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo.ops._native import available, native


def ceil16(v):
    return (int(v) + 15) // 16 * 16


def quantize_weight(w2):
    """[N, K] float -> (int8 [N, ceil16(K)], fp32 scale [N])."""
    w2 = w2.detach().float()
    N, K = w2.shape
    scale = w2.abs().amax(dim=1).clamp_min(1e-12) / 127.0
    q = torch.round(w2 / scale[:, None]).clamp_(-127, 127).to(torch.int8)
    out = torch.zeros(N, ceil16(K), dtype=torch.int8, device=w2.device)
    out[:, :K] = q
    return out, scale


def _q_act_ref(x, amax):
    inv = 127.0 / amax if amax > 0 else 0.0
    return torch.round((x.double() * inv).clamp(-127, 127))


def _im2col_nhwc(x, R, S, stride, pad):
    """[N,H,W,C] -> [N*P*Q, R*S*C] with k = (r*S + s)*C + c."""
    N, H, W, C = x.shape
    xp = F.pad(x, (0, 0, pad[1], pad[1], pad[0], pad[0]))
    P = (H + 2 * pad[0] - R) // stride[0] + 1
    Q = (W + 2 * pad[1] - S) // stride[1] + 1
    cols = []
    for r in range(R):
        for s in range(S):
            cols.append(xp[:, r:r + stride[0] * (P - 1) + 1:stride[0], s:s + stride[1] * (Q - 1) + 1:stride[1], :])
    return torch.cat(cols, dim=3).reshape(N * P * Q, R * S * C), P, Q


def qconv_nhwc(x, qw, wscale, bias=None, kernel=(1, 1), stride=(1, 1), pad=(0, 0), resid=None, relu=False,
               out_f32=False):
    """int8 conv: x NHWC (bf16/fp32), qw int8 [K, Kp] (packed (r,s,c) order)."""
    R, S = kernel
    N, H, W, C = x.shape
    K, Kp = qw.shape
    P = (H + 2 * pad[0] - R) // stride[0] + 1
    Q = (W + 2 * pad[1] - S) // stride[1] + 1
    if x.is_cuda:
        C_ = native()
        x = x.contiguous()
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        amax = C_.absmax(x)
        a = C_.im2col_q8(x, amax, R, S, stride[0], stride[1], pad[0], pad[1], P, Q, Kp)
        r = None if resid is None else resid.to(torch.bfloat16).contiguous().reshape(N * P * Q, K)
        y = C_.qgemm(a, qw, amax, wscale, None if bias is None else bias.float().contiguous(), r, bool(relu),
                     bool(out_f32))
        return y.reshape(N, P, Q, K)
    # CPU reference: identical integer arithmetic in float64
    amax = float(x.abs().max()) if x.numel() else 0.0
    cols, P, Q = _im2col_nhwc(x.float(), R, S, stride, pad)
    qa = _q_act_ref(cols, amax)
    acc = qa @ qw[:, :cols.shape[1]].double().t()
    y = acc * (amax / 127.0) * wscale.double()[None, :]
    if bias is not None:
        y = y + bias.double()[None, :]
    if resid is not None:
        y = y + resid.reshape(N * P * Q, K).double()
    if relu:
        y = y.clamp_min(0)
    y = y.float().reshape(N, P, Q, K)
    return y if (out_f32 or x.dtype == torch.float32) else y.to(x.dtype)


def qlinear(x, qw, wscale, bias=None, relu=False, out_f32=True):
    lead = x.shape[:-1]
    y = qconv_nhwc(x.reshape(-1, 1, 1, x.shape[-1]), qw, wscale, bias, relu=relu, out_f32=out_f32)
    return y.reshape(*lead, qw.shape[0])


class QuantizedLinear(nn.Module):
    def __init__(self, weight, bias=None, out_features=None, relu=False):
        super().__init__()
        qw, s = quantize_weight(weight)
        self.register_buffer("qweight", qw)
        self.register_buffer("wscale", s)
        self.register_buffer("bias", None if bias is None else bias.detach().float().clone())
        self.out_features = out_features or weight.shape[0]
        self.relu = relu

    def forward(self, x):
        y = qlinear(x, self.qweight, self.wscale, self.bias, relu=self.relu, out_f32=True)
        return y if y.shape[-1] == self.out_features else y[..., :self.out_features].contiguous()


class QuantizedConvBN(nn.Module):
    """Eval-mode ResNet ConvBN with BatchNorm folded into the int8 weights."""

    def __init__(self, unit):
        super().__init__()
        inv = torch.rsqrt(unit.running_var.float() + unit.eps)
        g = unit.gamma.detach().float() * inv
        w = unit.weight.detach().float()[:, :unit.k * unit.k * unit.cin] * g[:, None]
        qw, s = quantize_weight(w)
        self.register_buffer("qweight", qw)
        self.register_buffer("wscale", s)
        self.register_buffer("bias", unit.beta.detach().float() - unit.running_mean.float() * g)
        self.k, self.stride, self.pad, self.relu = unit.k, unit.stride, unit.pad, unit.relu

    def forward(self, x, resid=None, **_):
        return qconv_nhwc(x, self.qweight, self.wscale, self.bias, (self.k, self.k), (self.stride, self.stride),
                          (self.pad, self.pad), resid=resid, relu=self.relu)


class QuantizedConv2d(nn.Module):
    """torch.nn.Conv2d (NCHW, groups=1, dilation=1) on the int8 path."""

    def __init__(self, conv):
        super().__init__()
        w4 = conv.weight.detach().float().permute(0, 2, 3, 1)  # K,R,S,C
        qw, s = quantize_weight(w4.reshape(w4.shape[0], -1))
        self.register_buffer("qweight", qw)
        self.register_buffer("wscale", s)
        self.register_buffer("bias", None if conv.bias is None else conv.bias.detach().float().clone())
        self.kernel, self.stride, self.padding = conv.kernel_size, conv.stride, conv.padding

    def forward(self, x):
        y = qconv_nhwc(x.permute(0, 2, 3, 1).contiguous(), self.qweight, self.wscale, self.bias, self.kernel,
                       self.stride, self.padding, out_f32=True)
        return y.permute(0, 3, 1, 2).contiguous().to(x.dtype)


def _quantizable_conv(m):
    return isinstance(m, nn.Conv2d) and m.groups == 1 and tuple(m.dilation) == (1, 1) and \
        isinstance(m.padding, tuple) and m.padding_mode == "zeros"


def quantize(model, calib_data=None, dtype="int8"):
    """Convert supported layers of ``model`` to int8 in place; returns the model (eval mode).
    With ``calib_data`` (an input batch) a zoo ResNet is instead returned as its calibrated
    static twin (zoo.ops.qresnet.Int8ResNet; the original model is left as is); ``dtype="fp8"``
    selects the OCP e4m3 twin (Fp8ResNet, fp8 matrix cores), which needs calibration data."""
    from zoo.models.image import resnet as R
    from zoo.pipeline.api.keras.layers.core import Dense as KDense
    model.eval()
    if dtype not in ("int8", "fp8"):
        raise ValueError("dtype must be 'int8' or 'fp8'")
    if dtype == "fp8" and (calib_data is None or not isinstance(model, R.ResNet)):
        raise ValueError("fp8 quantization is the calibrated static path: a zoo ResNet and calib_data")
    if calib_data is not None and isinstance(model, R.ResNet):
        from zoo.ops.qresnet import Fp8ResNet, Int8ResNet
        dev = next(model.parameters()).device
        q = (Fp8ResNet if dtype == "fp8" else Int8ResNet)(model, torch.as_tensor(calib_data).to(dev))
        q._zoo_quantized = True
        return q

    def convert(parent):
        for name, child in list(parent.named_children()):
            new = None
            if isinstance(child, R.ConvBN):
                new = QuantizedConvBN(child)
            elif isinstance(child, R.Dense):
                new = QuantizedLinear(child.weight, child.bias, out_features=child.cout)
            elif isinstance(child, nn.Linear):
                new = QuantizedLinear(child.weight, child.bias)
            elif _quantizable_conv(child):
                new = QuantizedConv2d(child)
            elif isinstance(child, KDense) and getattr(child, "weight", None) is not None:
                child._qlinear = QuantizedLinear(child.weight, child.bias)
                child._orig_call = child.call
                child.call = _quantized_dense_call(child)
            if new is not None:
                setattr(parent, name, new.to(_dev(child)))
            else:
                convert(child)

    convert(model)
    model._zoo_quantized = True
    return model


def _dev(m):
    for t in list(m.parameters()) + list(m.buffers()):
        return t.device
    return torch.device("cpu")


def _quantized_dense_call(layer):
    from zoo.pipeline.api.keras.layers.core import apply_activation

    def call(x):
        y = layer._qlinear.to(x.device)(x)
        return apply_activation(y, layer.activation) if layer.activation is not None else y
    return call


def is_quantized(model):
    return bool(getattr(model, "_zoo_quantized", False))


__all__ = ["quantize", "quantize_weight", "qconv_nhwc", "qlinear", "QuantizedLinear", "QuantizedConvBN",
           "QuantizedConv2d", "is_quantized", "ceil16", "native_available"]


def native_available():
    return available()
