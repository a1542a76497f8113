"""Image-classification backbones of the reference's ImageClassifier configs
(Zs/models/image/imageclassification/ImageClassificationConfig.scala:56-190:
alexnet, inception-v1, inception-v3, resnet-50, vgg-16/19, densenet-161,
squeezenet, mobilenet, mobilenet-v2).

``build(name)`` returns the framework's native NHWC bf16 implementation
(zoo.models.image.native_nets, zoo.models.image.resnet). The plain NCHW
``torch.nn`` definitions below are kept as the architecture reference
(``build(name, native=False)``) for parity tests.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _cbr(cin, cout, k, s=1, p=0, bn=True, groups=1):
    layers = [nn.Conv2d(cin, cout, k, s, p, groups=groups, bias=not bn)]
    if bn:
        layers.append(nn.BatchNorm2d(cout))
    layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


class VGG(nn.Module):
    CFG = {16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
           19: [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]}

    def __init__(self, depth=16, num_classes=1000):
        super().__init__()
        layers, c = [], 3
        for v in self.CFG[depth]:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=True)]
                c = v
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(nn.Flatten(), nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(),
                                        nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(), nn.Linear(4096, num_classes))

    def forward(self, x):
        return self.classifier(F.adaptive_avg_pool2d(self.features(x), 7))


class AlexNet(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 11, 4, 2), nn.ReLU(True), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(True), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(True), nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(True),
            nn.Conv2d(256, 256, 3, padding=1), nn.ReLU(True), nn.MaxPool2d(3, 2))
        self.classifier = nn.Sequential(nn.Flatten(), nn.Dropout(), nn.Linear(256 * 36, 4096), nn.ReLU(True),
                                        nn.Dropout(), nn.Linear(4096, 4096), nn.ReLU(True),
                                        nn.Linear(4096, num_classes))

    def forward(self, x):
        return self.classifier(F.adaptive_avg_pool2d(self.features(x), 6))


class _Fire(nn.Module):
    def __init__(self, cin, s, e1, e3):
        super().__init__()
        self.s = _cbr(cin, s, 1, bn=False)
        self.e1 = _cbr(s, e1, 1, bn=False)
        self.e3 = _cbr(s, e3, 3, p=1, bn=False)

    def forward(self, x):
        x = self.s(x)
        return torch.cat([self.e1(x), self.e3(x)], 1)


class SqueezeNet(nn.Module):
    """SqueezeNet 1.1."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 3, 2), nn.ReLU(True), nn.MaxPool2d(3, 2, ceil_mode=True),
            _Fire(64, 16, 64, 64), _Fire(128, 16, 64, 64), nn.MaxPool2d(3, 2, ceil_mode=True),
            _Fire(128, 32, 128, 128), _Fire(256, 32, 128, 128), nn.MaxPool2d(3, 2, ceil_mode=True),
            _Fire(256, 48, 192, 192), _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), _Fire(512, 64, 256, 256))
        self.classifier = nn.Sequential(nn.Dropout(0.5), nn.Conv2d(512, num_classes, 1), nn.ReLU(True),
                                        nn.AdaptiveAvgPool2d(1), nn.Flatten())

    def forward(self, x):
        return self.classifier(self.features(x))


class MobileNet(nn.Module):
    """MobileNet v1 (depthwise-separable)."""

    def __init__(self, num_classes=1000, width=1.0):
        super().__init__()
        cfg = [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2)] + [(512, 1)] * 5 + [(1024, 2), (1024, 1)]
        c = int(32 * width)
        layers = [_cbr(3, c, 3, 2, 1)]
        for out, s in cfg:
            o = int(out * width)
            layers += [_cbr(c, c, 3, s, 1, groups=c), _cbr(c, o, 1)]
            c = o
        self.features = nn.Sequential(*layers)
        self.fc = nn.Linear(c, num_classes)

    def forward(self, x):
        return self.fc(F.adaptive_avg_pool2d(self.features(x), 1).flatten(1))


class _InvRes(nn.Module):
    def __init__(self, cin, cout, s, t):
        super().__init__()
        h = cin * t
        self.use_res = s == 1 and cin == cout
        layers = ([_cbr(cin, h, 1)] if t != 1 else []) + [_cbr(h, h, 3, s, 1, groups=h),
                                                           nn.Conv2d(h, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
               (6, 320, 1, 1)]
        layers, c = [_cbr(3, 32, 3, 2, 1)], 32
        for t, o, n, s in cfg:
            for i in range(n):
                layers.append(_InvRes(c, o, s if i == 0 else 1, t))
                c = o
        layers.append(_cbr(c, 1280, 1))
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(1280, num_classes))

    def forward(self, x):
        return self.classifier(F.adaptive_avg_pool2d(self.features(x), 1).flatten(1))


class _Inception(nn.Module):
    def __init__(self, cin, c1, c3r, c3, c5r, c5, pp):
        super().__init__()
        self.b1 = _cbr(cin, c1, 1)
        self.b2 = nn.Sequential(_cbr(cin, c3r, 1), _cbr(c3r, c3, 3, p=1))
        self.b3 = nn.Sequential(_cbr(cin, c5r, 1), _cbr(c5r, c5, 3, p=1))
        self.b4 = nn.Sequential(nn.MaxPool2d(3, 1, 1), _cbr(cin, pp, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b2(x), self.b3(x), self.b4(x)], 1)


class InceptionV1(nn.Module):
    """GoogLeNet (BN variant, no auxiliary heads at inference)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(_cbr(3, 64, 7, 2, 3), nn.MaxPool2d(3, 2, ceil_mode=True), _cbr(64, 64, 1),
                                  _cbr(64, 192, 3, p=1), nn.MaxPool2d(3, 2, ceil_mode=True))
        self.blocks = nn.Sequential(
            _Inception(192, 64, 96, 128, 16, 32, 32), _Inception(256, 128, 128, 192, 32, 96, 64),
            nn.MaxPool2d(3, 2, ceil_mode=True),
            _Inception(480, 192, 96, 208, 16, 48, 64), _Inception(512, 160, 112, 224, 24, 64, 64),
            _Inception(512, 128, 128, 256, 24, 64, 64), _Inception(512, 112, 144, 288, 32, 64, 64),
            _Inception(528, 256, 160, 320, 32, 128, 128), nn.MaxPool2d(2, 2, ceil_mode=True),
            _Inception(832, 256, 160, 320, 32, 128, 128), _Inception(832, 384, 192, 384, 48, 128, 128))
        self.fc = nn.Sequential(nn.Dropout(0.4), nn.Linear(1024, num_classes))

    def forward(self, x):
        return self.fc(F.adaptive_avg_pool2d(self.blocks(self.stem(x)), 1).flatten(1))


class _DenseLayer(nn.Module):
    def __init__(self, cin, growth, bn_size):
        super().__init__()
        self.net = nn.Sequential(nn.BatchNorm2d(cin), nn.ReLU(True), nn.Conv2d(cin, bn_size * growth, 1, bias=False),
                                 nn.BatchNorm2d(bn_size * growth), nn.ReLU(True),
                                 nn.Conv2d(bn_size * growth, growth, 3, padding=1, bias=False))

    def forward(self, x):
        return torch.cat([x, self.net(x)], 1)


class DenseNet(nn.Module):
    """DenseNet-161 by default (growth 48, blocks 6-12-36-24)."""

    def __init__(self, num_classes=1000, growth=48, blocks=(6, 12, 36, 24), init_features=96, bn_size=4):
        super().__init__()
        layers = [nn.Conv2d(3, init_features, 7, 2, 3, bias=False), nn.BatchNorm2d(init_features), nn.ReLU(True),
                  nn.MaxPool2d(3, 2, 1)]
        c = init_features
        for i, n in enumerate(blocks):
            for _ in range(n):
                layers.append(_DenseLayer(c, growth, bn_size))
                c += growth
            if i != len(blocks) - 1:
                layers += [nn.BatchNorm2d(c), nn.ReLU(True), nn.Conv2d(c, c // 2, 1, bias=False), nn.AvgPool2d(2, 2)]
                c //= 2
        layers += [nn.BatchNorm2d(c), nn.ReLU(True)]
        self.features = nn.Sequential(*layers)
        self.fc = nn.Linear(c, num_classes)

    def forward(self, x):
        return self.fc(F.adaptive_avg_pool2d(self.features(x), 1).flatten(1))


class _IncA(nn.Module):
    def __init__(self, cin, pool):
        super().__init__()
        self.b1 = _cbr(cin, 64, 1)
        self.b5 = nn.Sequential(_cbr(cin, 48, 1), _cbr(48, 64, 5, p=2))
        self.b3 = nn.Sequential(_cbr(cin, 64, 1), _cbr(64, 96, 3, p=1), _cbr(96, 96, 3, p=1))
        self.bp = nn.Sequential(nn.AvgPool2d(3, 1, 1), _cbr(cin, pool, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b5(x), self.b3(x), self.bp(x)], 1)


class InceptionV3(nn.Module):
    """Inception-v3 (stem + A blocks + grid reductions; compact B/C stages)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(_cbr(3, 32, 3, 2), _cbr(32, 32, 3), _cbr(32, 64, 3, p=1), nn.MaxPool2d(3, 2),
                                  _cbr(64, 80, 1), _cbr(80, 192, 3), nn.MaxPool2d(3, 2))
        self.a = nn.Sequential(_IncA(192, 32), _IncA(256, 64), _IncA(288, 64))
        self.red1 = _cbr(288, 768, 3, 2)
        self.b = nn.Sequential(*[nn.Sequential(_cbr(768, 192, 1), _cbr(192, 192, (1, 7), p=(0, 3)),
                                               _cbr(192, 768, (7, 1), p=(3, 0))) for _ in range(4)])
        self.red2 = _cbr(768, 1280, 3, 2)
        self.c = nn.Sequential(_cbr(1280, 2048, 1), _cbr(2048, 2048, 3, p=1, groups=16))
        self.fc = nn.Sequential(nn.Dropout(0.5), nn.Linear(2048, num_classes))

    def forward(self, x):
        x = self.a(self.stem(x))
        x = self.red1(x)
        for blk in self.b:
            x = x + blk(x)
        x = self.c(self.red2(x))
        return self.fc(F.adaptive_avg_pool2d(x, 1).flatten(1))


def build(name, num_classes=1000, native=True):
    n = name.lower()
    if n in ("resnet-50", "resnet-50-int8", "resnet-50-quantize"):
        from zoo.models.image.resnet import resnet50
        return resnet50(num_classes=num_classes)
    if native:
        from zoo.models.image.native_nets import TABLE
        for k in sorted(TABLE, key=len, reverse=True):
            if n.startswith(k):
                return TABLE[k](num_classes)
    table = {"vgg-16": lambda: VGG(16, num_classes), "vgg-19": lambda: VGG(19, num_classes),
             "alexnet": lambda: AlexNet(num_classes), "squeezenet": lambda: SqueezeNet(num_classes),
             "mobilenet": lambda: MobileNet(num_classes), "mobilenet-v2": lambda: MobileNetV2(num_classes),
             "inception-v1": lambda: InceptionV1(num_classes), "inception-v3": lambda: InceptionV3(num_classes),
             "densenet-161": lambda: DenseNet(num_classes)}
    for k, f in table.items():
        if n.startswith(k):
            return f()
    raise ValueError("unknown image classification model %s (known: resnet-50, %s)" % (name, ", ".join(table)))
