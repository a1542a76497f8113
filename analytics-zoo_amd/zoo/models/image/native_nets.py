"""The ImageClassifier backbones (Zs/models/image/imageclassification/
ImageClassificationConfig.scala:56-190: alexnet, vgg-16/19, squeezenet,
mobilenet, mobilenet-v2, inception-v1, inception-v3, densenet-161) built from
the framework's native NHWC bf16 units instead of ``torch.nn`` / MIOpen:

  * ``CBR``   conv (implicit-GEMM MFMA kernel) + BatchNorm (statistics in the
              conv epilogue) + ReLU -- ``ops.conv_bn_act``
  * ``CB``    conv + bias + ReLU fused in the GEMM epilogue (AlexNet / VGG /
              SqueezeNet have no BN) -- ``ops.conv2d_nhwc``
  * ``DWBR``  depthwise conv (dwconv.hip) + native BatchNorm(+ReLU)
  * pooling   native NHWC max / average / global-average pooling
  * ``Dense`` the MFMA GEMM with fp32 logits

Activations stay NHWC bf16 from the input conversion to the classifier; branch
concatenation is a channel-dim ``torch.cat`` of NHWC tensors. On CPU every unit
runs its PyTorch reference (the same code path the CPU tests use).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.models.image.resnet import Dense


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def to_nhwc(x, cin, cin_pad):
    """NCHW fp32 images ([N, cin, H, W]) -> NHWC bf16 with channels zero-padded to
    ``cin_pad``; anything else is taken to be NHWC already."""
    if x.dim() == 4 and x.shape[1] == cin and x.shape[-1] != cin_pad:
        if x.is_cuda:
            return ops.native().nchw_to_nhwc(x.float().contiguous(), cin_pad)
        x = x.permute(0, 2, 3, 1)
        pad = cin_pad - x.shape[-1]
        if pad:
            x = F.pad(x, (0, pad))
        return x.contiguous()
    return x


def _cin_pad(c):
    return 4 if c <= 4 else ops.ceil8(c)


class CBR(nn.Module):
    """conv(KhxKw) -> BatchNorm -> ReLU on NHWC (packed [K, ceil8(R*S*C)] weight)."""

    def __init__(self, cin, cout, k, stride=1, pad=0, relu=True):
        super().__init__()
        self.k, self.stride, self.pad = _pair(k), _pair(stride), _pair(pad)
        self.relu = relu
        R, S = self.k
        w4 = torch.empty(cout, R, S, cin)
        nn.init.normal_(w4, 0.0, math.sqrt(2.0 / (cout * R * S)))
        self.weight = nn.Parameter(ops.pack_weight(w4))
        self.gamma = nn.Parameter(torch.ones(cout))
        self.beta = nn.Parameter(torch.zeros(cout))
        self.register_buffer("running_mean", torch.zeros(cout))
        self.register_buffer("running_var", torch.ones(cout))

    def forward(self, x, resid=None):
        return ops.conv_bn_act(x, self.weight, self.gamma, self.beta, self.running_mean, self.running_var,
                               kernel=self.k, stride=self.stride, pad=self.pad, relu=self.relu, resid=resid,
                               training=self.training)


class CB(nn.Module):
    """conv + bias (+ ReLU) fused in the GEMM epilogue (no BatchNorm). Output channels
    are padded to a multiple of 8 for the MFMA kernel (the padded filters stay zero:
    they only ever receive zero gradient) and sliced off."""

    def __init__(self, cin, cout, k, stride=1, pad=0, relu=True, dil=1):
        super().__init__()
        self.k, self.stride, self.pad, self.relu = _pair(k), _pair(stride), _pair(pad), relu
        self.dil, self.cout = _pair(dil), cout
        R, S = self.k
        kp = ops.ceil8(cout)
        w4 = torch.zeros(kp, R, S, cin)
        nn.init.kaiming_uniform_(w4[:cout].view(cout, -1), a=math.sqrt(5))
        self.weight = nn.Parameter(ops.pack_weight(w4))
        self.bias = nn.Parameter(torch.zeros(kp))

    def forward(self, x):
        y = ops.conv2d_nhwc(x, self.weight, self.bias, kernel=self.k, stride=self.stride, pad=self.pad, dil=self.dil,
                            act="relu" if self.relu else None)
        return y if y.shape[-1] == self.cout else y[..., :self.cout]


class DWBR(nn.Module):
    """depthwise conv -> BatchNorm -> ReLU (MobileNet units)."""

    def __init__(self, c, k=3, stride=1, pad=1, relu=True):
        super().__init__()
        self.k, self.stride, self.pad, self.relu = _pair(k), _pair(stride), _pair(pad), relu
        self.weight = nn.Parameter(torch.randn(self.k[0] * self.k[1], c) * math.sqrt(2.0 / (self.k[0] * self.k[1])))
        self.gamma = nn.Parameter(torch.ones(c))
        self.beta = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))

    def forward(self, x):
        from zoo.ops.nn import depthwise_bn_act_eval, depthwise_conv2d_nhwc
        if x.is_cuda and not self.training and not torch.is_grad_enabled() and x.shape[-1] % 8 == 0 and \
                self.k[0] * self.k[1] <= 9:
            return depthwise_bn_act_eval(x, self.weight, self.gamma, self.beta, self.running_mean, self.running_var,
                                         self.k, self.stride, self.pad, relu=self.relu)
        y = depthwise_conv2d_nhwc(x, self.weight, None, self.k, self.stride, self.pad)
        return ops.batch_norm_nhwc(y, self.gamma, self.beta, self.running_mean, self.running_var, relu=self.relu,
                                   training=self.training)


class BNR(nn.Module):
    """standalone BatchNorm (+ReLU) (DenseNet pre-activation)."""

    def __init__(self, c, relu=True):
        super().__init__()
        self.relu = relu
        self.gamma = nn.Parameter(torch.ones(c))
        self.beta = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))

    def forward(self, x):
        return ops.batch_norm_nhwc(x, self.gamma, self.beta, self.running_mean, self.running_var, relu=self.relu,
                                   training=self.training)


class MaxPool(nn.Module):
    def __init__(self, k, s=None, p=0, ceil_mode=False):
        super().__init__()
        self.k, self.s, self.p, self.ceil = _pair(k), _pair(s or k), _pair(p), ceil_mode

    def forward(self, x):
        return ops.max_pool2d_nhwc(x, self.k, self.s, self.p, ceil_mode=self.ceil)


class AvgPool(nn.Module):
    def __init__(self, k, s=None, p=0, ceil_mode=False, count_include_pad=True):
        super().__init__()
        self.k, self.s, self.p = _pair(k), _pair(s or k), _pair(p)
        self.ceil, self.inc = ceil_mode, count_include_pad

    def forward(self, x):
        from zoo.ops.pool import avg_pool2d_nhwc
        return avg_pool2d_nhwc(x, self.k, self.s, self.p, ceil_mode=self.ceil, count_include_pad=self.inc)


def gap(x):
    return ops.global_avg_pool_nhwc(x)


def cat(xs):
    return torch.cat(xs, dim=-1)


def _dropout(x, p, training):
    return F.dropout(x, p, training) if training and p > 0 else x


class NativeNet(nn.Module):
    """Base: NCHW fp32 input -> NHWC bf16 -> features -> classifier. ``trace_hw``: the input
    size the BigDL graph encoder (zoo.utils.bigdl_graph.native_graph_spec) traces at."""

    in_channels = 3
    trace_hw = 224

    def prepare(self, x):
        return to_nhwc(x, self.in_channels, _cin_pad(self.in_channels))


# ---------------------------------------------------------------------------
class VGG(NativeNet):
    CFG = {16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
           19: [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512,
                "M"]}

    def __init__(self, depth=16, num_classes=1000):
        super().__init__()
        layers, c = [], _cin_pad(3)
        for v in self.CFG[depth]:
            if v == "M":
                layers.append(MaxPool(2, 2))
            else:
                layers.append(CB(c, v, 3, 1, 1))
                c = v
        self.features = nn.Sequential(*layers)
        self.fc1, self.fc2, self.fc3 = Dense(512 * 7 * 7, 4096), Dense(4096, 4096), Dense(4096, num_classes)

    def forward(self, x):
        h = self.features(self.prepare(x))
        if h.shape[1] != 7:
            h = F.adaptive_avg_pool2d(h.permute(0, 3, 1, 2).float(), 7).permute(0, 2, 3, 1)
        h = h.reshape(h.shape[0], -1)
        h = _dropout(torch.relu(self.fc1(h)), 0.5, self.training)
        h = _dropout(torch.relu(self.fc2(h)), 0.5, self.training)
        return self.fc3(h)


class AlexNet(NativeNet):
    trace_hw = 227

    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            CB(_cin_pad(3), 64, 11, 4, 2), MaxPool(3, 2), CB(64, 192, 5, 1, 2), MaxPool(3, 2),
            CB(192, 384, 3, 1, 1), CB(384, 256, 3, 1, 1), CB(256, 256, 3, 1, 1), MaxPool(3, 2))
        self.fc1, self.fc2, self.fc3 = Dense(256 * 36, 4096), Dense(4096, 4096), Dense(4096, num_classes)

    def forward(self, x):
        h = self.features(self.prepare(x))
        if h.shape[1] != 6:
            h = F.adaptive_avg_pool2d(h.permute(0, 3, 1, 2).float(), 6).permute(0, 2, 3, 1)
        h = h.reshape(h.shape[0], -1)
        h = torch.relu(self.fc1(_dropout(h, 0.5, self.training)))
        h = torch.relu(self.fc2(_dropout(h, 0.5, self.training)))
        return self.fc3(h)


class _Fire(nn.Module):
    def __init__(self, cin, s, e1, e3):
        super().__init__()
        self.s, self.e1, self.e3 = CB(cin, s, 1), CB(s, e1, 1), CB(s, e3, 3, 1, 1)

    def forward(self, x):
        x = self.s(x)
        return cat([self.e1(x), self.e3(x)])


class SqueezeNet(NativeNet):
    """SqueezeNet 1.1."""

    trace_hw = 227

    def __init__(self, num_classes=1000):
        super().__init__()
        self.num_classes = num_classes
        self.features = nn.Sequential(
            CB(_cin_pad(3), 64, 3, 2), MaxPool(3, 2, ceil_mode=True),
            _Fire(64, 16, 64, 64), _Fire(128, 16, 64, 64), MaxPool(3, 2, ceil_mode=True),
            _Fire(128, 32, 128, 128), _Fire(256, 32, 128, 128), MaxPool(3, 2, ceil_mode=True),
            _Fire(256, 48, 192, 192), _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), _Fire(512, 64, 256, 256))
        self.head = CB(512, ops.ceil8(num_classes), 1)

    def forward(self, x):
        h = self.head(_dropout(self.features(self.prepare(x)), 0.5, self.training))
        return gap(h).float()[:, :self.num_classes]


class MobileNet(NativeNet):
    """MobileNet v1 (depthwise-separable)."""

    def __init__(self, num_classes=1000, width=1.0):
        super().__init__()
        cfg = [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2)] + [(512, 1)] * 5 + [(1024, 2), (1024, 1)]
        c = int(32 * width)
        layers = [CBR(_cin_pad(3), c, 3, 2, 1)]
        for out, s in cfg:
            o = int(out * width)
            layers += [DWBR(c, 3, s, 1), CBR(c, o, 1)]
            c = o
        self.features = nn.Sequential(*layers)
        self.fc = Dense(c, num_classes)

    def forward(self, x):
        return self.fc(gap(self.features(self.prepare(x))))


class _InvRes(nn.Module):
    def __init__(self, cin, cout, s, t):
        super().__init__()
        h = cin * t
        self.use_res = s == 1 and cin == cout
        self.expand = CBR(cin, h, 1) if t != 1 else None
        self.dw = DWBR(h, 3, s, 1)
        self.project = CBR(h, cout, 1, relu=False)

    def forward(self, x):
        h = self.expand(x) if self.expand is not None else x
        return self.project(self.dw(h), resid=x if self.use_res else None)


class MobileNetV2(NativeNet):
    def __init__(self, num_classes=1000):
        super().__init__()
        cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
               (6, 320, 1, 1)]
        layers, c = [CBR(_cin_pad(3), 32, 3, 2, 1)], 32
        for t, o, n, s in cfg:
            for i in range(n):
                layers.append(_InvRes(c, o, s if i == 0 else 1, t))
                c = o
        layers.append(CBR(c, 1280, 1))
        self.features = nn.Sequential(*layers)
        self.fc = Dense(1280, num_classes)

    def forward(self, x):
        return self.fc(_dropout(gap(self.features(self.prepare(x))), 0.2, self.training))


class _Inception(nn.Module):
    def __init__(self, cin, c1, c3r, c3, c5r, c5, pp):
        super().__init__()
        self.b1 = CBR(cin, c1, 1)
        self.b2 = nn.Sequential(CBR(cin, c3r, 1), CBR(c3r, c3, 3, 1, 1))
        self.b3 = nn.Sequential(CBR(cin, c5r, 1), CBR(c5r, c5, 3, 1, 1))
        self.pool = MaxPool(3, 1, 1)
        self.b4 = CBR(cin, pp, 1)

    def forward(self, x):
        return cat([self.b1(x), self.b2(x), self.b3(x), self.b4(self.pool(x))])


class InceptionV1(NativeNet):
    """GoogLeNet (BN variant)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(CBR(_cin_pad(3), 64, 7, 2, 3), MaxPool(3, 2, ceil_mode=True), CBR(64, 64, 1),
                                  CBR(64, 192, 3, 1, 1), MaxPool(3, 2, ceil_mode=True))
        self.blocks = nn.Sequential(
            _Inception(192, 64, 96, 128, 16, 32, 32), _Inception(256, 128, 128, 192, 32, 96, 64),
            MaxPool(3, 2, ceil_mode=True),
            _Inception(480, 192, 96, 208, 16, 48, 64), _Inception(512, 160, 112, 224, 24, 64, 64),
            _Inception(512, 128, 128, 256, 24, 64, 64), _Inception(512, 112, 144, 288, 32, 64, 64),
            _Inception(528, 256, 160, 320, 32, 128, 128), MaxPool(2, 2, ceil_mode=True),
            _Inception(832, 256, 160, 320, 32, 128, 128), _Inception(832, 384, 192, 384, 48, 128, 128))
        self.fc = Dense(1024, num_classes)

    def forward(self, x):
        return self.fc(_dropout(gap(self.blocks(self.stem(self.prepare(x)))), 0.4, self.training))


class _DenseLayer(nn.Module):
    def __init__(self, cin, growth, bn_size):
        super().__init__()
        self.bn = BNR(cin)
        self.conv1 = CBR(cin, bn_size * growth, 1)      # conv -> BN -> ReLU of the bottleneck
        self.conv2 = CB(bn_size * growth, growth, 3, 1, 1, relu=False)

    def forward(self, x):
        return cat([x, self.conv2(self.conv1(self.bn(x)))])


class DenseNet(NativeNet):
    """DenseNet-161 by default (growth 48, blocks 6-12-36-24)."""

    def __init__(self, num_classes=1000, growth=48, blocks=(6, 12, 36, 24), init_features=96, bn_size=4):
        super().__init__()
        layers = [CBR(_cin_pad(3), init_features, 7, 2, 3), MaxPool(3, 2, 1)]
        c = init_features
        for i, n in enumerate(blocks):
            for _ in range(n):
                layers.append(_DenseLayer(c, growth, bn_size))
                c += growth
            if i != len(blocks) - 1:
                layers += [BNR(c), CB(c, c // 2, 1, relu=False), AvgPool(2, 2)]
                c //= 2
        layers.append(BNR(c))
        self.features = nn.Sequential(*layers)
        self.fc = Dense(c, num_classes)

    def forward(self, x):
        return self.fc(gap(self.features(self.prepare(x))))


class _IncA(nn.Module):
    def __init__(self, cin, pool):
        super().__init__()
        self.b1 = CBR(cin, 64, 1)
        self.b5 = nn.Sequential(CBR(cin, 48, 1), CBR(48, 64, 5, 1, 2))
        self.b3 = nn.Sequential(CBR(cin, 64, 1), CBR(64, 96, 3, 1, 1), CBR(96, 96, 3, 1, 1))
        self.pool = AvgPool(3, 1, 1)
        self.bp = CBR(cin, pool, 1)

    def forward(self, x):
        return cat([self.b1(x), self.b5(x), self.b3(x), self.bp(self.pool(x))])


class InceptionV3(NativeNet):
    """Inception-v3 (stem + A blocks + grid reductions; factorised 1x7/7x1 B stage)."""

    trace_hw = 299

    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(CBR(_cin_pad(3), 32, 3, 2), CBR(32, 32, 3), CBR(32, 64, 3, 1, 1), MaxPool(3, 2),
                                  CBR(64, 80, 1), CBR(80, 192, 3), MaxPool(3, 2))
        self.a = nn.Sequential(_IncA(192, 32), _IncA(256, 64), _IncA(288, 64))
        self.red1 = CBR(288, 768, 3, 2)
        self.b = nn.ModuleList([nn.Sequential(CBR(768, 192, 1), CBR(192, 192, (1, 7), 1, (0, 3)),
                                              CBR(192, 768, (7, 1), 1, (3, 0), relu=False)) for _ in range(4)])
        self.red2 = CBR(768, 1280, 3, 2)
        self.c = nn.Sequential(CBR(1280, 2048, 1), CBR(2048, 2048, 3, 1, 1))
        self.fc = Dense(2048, num_classes)

    def forward(self, x):
        x = self.red1(self.a(self.stem(self.prepare(x))))
        for blk in self.b:
            x = torch.relu(x + blk(x))
        x = self.c(self.red2(x))
        return self.fc(_dropout(gap(x), 0.5, self.training))


TABLE = {"vgg-16": lambda n: VGG(16, n), "vgg-19": lambda n: VGG(19, n), "alexnet": AlexNet,
         "squeezenet": SqueezeNet, "mobilenet-v2": MobileNetV2, "mobilenet": MobileNet,
         "inception-v1": InceptionV1, "inception-v3": InceptionV3, "densenet-161": DenseNet}
