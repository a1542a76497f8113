"""Faster R-CNN (the reference's "frcnn-vgg16" / "frcnn-pvanet" ObjectDetector
configs: Zs/models/image/objectdetection/ObjectDetectionConfig.scala:38-46, 70-135;
post-processing Postprocessor.scala:30-75; BigDL Proposal / RoiPooling /
DetectionOutputFrcnn layers behind them).

On the GPU the whole network runs channels-last on the native kernels: backbone
(VGG16 conv1-conv5 / PVANet) and RPN convolutions on the implicit-GEMM MFMA conv with the
bias + ReLU epilogue, max pooling, PVANet's C.ReLU BatchNorm and hyper-feature resize on the
NHWC kernels, RoI max pooling on its own kernel (csrc/kernels/roi.hip), the fc heads on the
framework's linear op. The parameters stay in torch layout (nn.Conv2d / nn.Linear) so the
reference's weights load unchanged; the packed bf16 conv weights are derived and cached per
weight version. On the CPU the same modules run as the fp32 torch reference. Proposal
generation and per-class detection output are vectorised on the device; only the greedy NMS
loop runs on the host, as in SSD's DetectionOutput.

Pre-processing follows ``preprocessFrcnn(resolution, scaleMultipleOf)``: aspect
scale to ``resolution`` on the short side (600 for VGG16, 640 with multiples of
32 for PVANet), BGR mean subtraction (122.7717, 115.9465, 102.9801), and an
``im_info`` = (height, width, scale) tensor per image.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.models.image.objectdetection.ssd import nms

FRCNN_MEANS = (122.7717, 115.9465, 102.9801)


def generate_anchors(base_size=16, ratios=(0.5, 1.0, 2.0), scales=(8, 16, 32)):
    """The 9 reference anchors (x1, y1, x2, y2) centred on one ``base_size`` cell."""
    ctr = (base_size - 1) / 2.0
    out = []
    for r in ratios:
        size = base_size * base_size / r
        ws = round(math.sqrt(size))
        hs = round(ws * r)
        for s in scales:
            w, h = ws * s, hs * s
            out.append([ctr - (w - 1) / 2, ctr - (h - 1) / 2, ctr + (w - 1) / 2, ctr + (h - 1) / 2])
    return torch.tensor(out, dtype=torch.float32)


def bbox_transform_inv(boxes, deltas):
    """Apply (dx, dy, dw, dh) regression deltas to pixel boxes."""
    w = boxes[:, 2] - boxes[:, 0] + 1.0
    h = boxes[:, 3] - boxes[:, 1] + 1.0
    cx = boxes[:, 0] + 0.5 * w
    cy = boxes[:, 1] + 0.5 * h
    dx, dy, dw, dh = deltas[:, 0::4], deltas[:, 1::4], deltas[:, 2::4], deltas[:, 3::4]
    pcx = dx * w[:, None] + cx[:, None]
    pcy = dy * h[:, None] + cy[:, None]
    pw = torch.exp(dw.clamp(max=math.log(1000.0 / 16))) * w[:, None]
    ph = torch.exp(dh.clamp(max=math.log(1000.0 / 16))) * h[:, None]
    out = torch.empty_like(deltas)
    out[:, 0::4] = pcx - 0.5 * pw
    out[:, 1::4] = pcy - 0.5 * ph
    out[:, 2::4] = pcx + 0.5 * pw - 1
    out[:, 3::4] = pcy + 0.5 * ph - 1
    return out


def clip_boxes(boxes, h, w):
    boxes[:, 0::4] = boxes[:, 0::4].clamp(0, w - 1)
    boxes[:, 1::4] = boxes[:, 1::4].clamp(0, h - 1)
    boxes[:, 2::4] = boxes[:, 2::4].clamp(0, w - 1)
    boxes[:, 3::4] = boxes[:, 3::4].clamp(0, h - 1)
    return boxes


class Proposal(nn.Module):
    """RPN scores + deltas -> RoIs [R, 5] (batch index, x1, y1, x2, y2)."""

    def __init__(self, pre_nms_topn=6000, post_nms_topn=300, nms_thresh=0.7, min_size=16, feat_stride=16,
                 ratios=(0.5, 1.0, 2.0), scales=(8, 16, 32)):
        super().__init__()
        self.pre, self.post, self.thresh, self.min_size, self.stride = pre_nms_topn, post_nms_topn, nms_thresh, \
            min_size, feat_stride
        self.register_buffer("anchors", generate_anchors(feat_stride, ratios, scales))

    @torch.no_grad()
    def forward(self, cls_prob, bbox_deltas, im_info):
        B, twoA, H, W = cls_prob.shape
        A = twoA // 2
        dev = cls_prob.device
        sx = torch.arange(W, device=dev, dtype=torch.float32) * self.stride
        sy = torch.arange(H, device=dev, dtype=torch.float32) * self.stride
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        shifts = torch.stack([xx, yy, xx, yy], -1).reshape(-1, 1, 4)                 # [HW, 1, 4]
        all_anchors = (self.anchors.to(dev)[None] + shifts).reshape(-1, 4)          # [HW*A, 4]
        rois = []
        for b in range(B):
            scores = cls_prob[b, A:].permute(1, 2, 0).reshape(-1)                   # foreground probs
            deltas = bbox_deltas[b].permute(1, 2, 0).reshape(-1, 4)
            props = clip_boxes(bbox_transform_inv(all_anchors, deltas.float()), float(im_info[b, 0]),
                               float(im_info[b, 1]))
            ms = self.min_size * float(im_info[b, 2])
            keep = ((props[:, 2] - props[:, 0] + 1) >= ms) & ((props[:, 3] - props[:, 1] + 1) >= ms)
            props, scores = props[keep], scores[keep].float()
            order = scores.argsort(descending=True)[:self.pre]
            props, scores = props[order], scores[order]
            k = nms(props, scores, self.thresh, props.shape[0], max_keep=self.post)[:self.post]
            rois.append(torch.cat([torch.full((k.numel(), 1), float(b), device=dev), props[k]], 1))
        return torch.cat(rois) if rois else torch.zeros(0, 5, device=dev)


def roi_pool(features, rois, pooled=7, spatial_scale=1.0 / 16, return_argmax=False):
    """Max RoI pooling (BigDL RoiPooling / Caffe ROIPooling) of NCHW features: each RoI is
    rounded to feature coordinates and split into pooled x pooled fractional bins
    [floor(i * h / P), ceil((i + 1) * h / P)), clipped to the map; an empty bin is 0.
    fp32 reference of the native channels-last kernel (roi_pool_nhwc). ``return_argmax``
    also returns the Caffe argmax (flat h * W + w of the FIRST maximum in row-major order,
    -1 for an empty bin) that routes the backward; autograd through ``amax`` would split the
    gradient between tied maxima instead."""
    out = features.new_zeros(rois.shape[0], features.shape[1], pooled, pooled)
    arg = torch.full(out.shape, -1, dtype=torch.long, device=features.device) if return_argmax else None
    H, W = features.shape[2], features.shape[3]
    # C round() (half away from zero) of the fp32 scaled box, bin edges in fp32 arithmetic --
    # exactly what Caffe's ROIPoolingLayer (and the native kernel) compute
    v = (rois[:, 1:].float() * np.float32(spatial_scale)).cpu().numpy().astype(np.float32)
    r = (np.sign(v) * np.floor(np.abs(v) + np.float32(0.5))).astype(np.int64).tolist()
    bidx = rois[:, 0].long().clamp(0, features.shape[0] - 1).tolist()
    P = np.float32(pooled)
    for i in range(rois.shape[0]):
        x1, y1, x2, y2 = r[i]
        rw, rh = max(x2 - x1 + 1, 1), max(y2 - y1 + 1, 1)
        bw, bh = np.float32(rw) / P, np.float32(rh) / P
        for ph in range(pooled):
            hs = min(max(int(np.floor(np.float32(ph) * bh)) + y1, 0), H)
            he = min(max(int(np.ceil(np.float32(ph + 1) * bh)) + y1, 0), H)
            for pw in range(pooled):
                ws = min(max(int(np.floor(np.float32(pw) * bw)) + x1, 0), W)
                we = min(max(int(np.ceil(np.float32(pw + 1) * bw)) + x1, 0), W)
                if hs < he and ws < we:
                    win = features[bidx[i], :, hs:he, ws:we]
                    out[i, :, ph, pw] = win.amax((1, 2))
                    if arg is not None:
                        a = win.detach().flatten(1).argmax(1)      # first maximum
                        arg[i, :, ph, pw] = (hs + a // (we - ws)) * W + ws + a % (we - ws)
    return (out, arg) if return_argmax else out


class _RoiPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, rois, pooled, scale):
        out, arg = ops.native().roi_pool_fwd(f, rois, pooled, pooled, scale)
        ctx.save_for_backward(arg, rois)
        ctx.fshape = f.shape
        return out

    @staticmethod
    def backward(ctx, dy):
        arg, rois = ctx.saved_tensors
        B, H, W, _ = ctx.fshape
        df = ops.native().roi_pool_bwd(dy.contiguous(), arg, rois, B, H, W)
        return df, None, None, None


def roi_pool_nhwc(features, rois, pooled=7, spatial_scale=1.0 / 16):
    """Native max RoI pooling of channels-last features -> [R, pooled, pooled, C]."""
    return _RoiPoolFn.apply(features.contiguous(), rois.float().contiguous(), int(pooled), float(spatial_scale))


def _packed_conv(conv, cin):
    """nn.Conv2d [K, C, R, S] -> packed [ceil8(K), ldb] weight over ``cin`` (>= C, zero padded)
    input channels plus the padded bias; cached on the module per weight version."""
    key = (conv.weight._version, conv.weight.data_ptr(), cin,
           None if conv.bias is None else (conv.bias._version, conv.bias.data_ptr()))
    c = getattr(conv, "_zoo_packed", None)
    if c is not None and c[0] == key and not torch.is_grad_enabled():
        return c[1], c[2]
    K, C, R, S = conv.weight.shape
    w4 = F.pad(conv.weight.permute(0, 2, 3, 1), (0, cin - C, 0, 0, 0, 0, 0, ops.ceil8(K) - K))
    wp = ops.pack_weight(w4)
    b = None if conv.bias is None else F.pad(conv.bias, (0, ops.ceil8(K) - K))
    if not torch.is_grad_enabled():
        conv._zoo_packed = (key, wp, b)
    return wp, b


def _nconv(x, conv, act=None):
    """NHWC conv on the implicit-GEMM kernel with the module's own stride / padding."""
    C = x.shape[-1]
    wp, b = _packed_conv(conv, C)
    y = ops.conv2d_nhwc(x, wp, b, kernel=conv.kernel_size, stride=conv.stride, pad=conv.padding, act=act)
    K = conv.out_channels
    return y if y.shape[-1] == K else y[..., :K]


class DetectionOutputFrcnn(nn.Module):
    """Per-class box decode + NMS -> per-image [K, 6] (label, score, x1, y1, x2, y2)
    in input-image pixels divided by the scale (i.e. original-image pixels)."""

    def __init__(self, num_classes=21, nms_thresh=0.3, max_per_image=100, thresh=0.05, bg_label=0):
        super().__init__()
        self.n, self.nms_thresh, self.max_per_image, self.thresh, self.bg = num_classes, nms_thresh, \
            max_per_image, thresh, bg_label

    @torch.no_grad()
    def forward(self, rois, cls_prob, bbox_pred, im_info):
        out = []
        B = im_info.shape[0]
        for b in range(B):
            sel = rois[:, 0] == b
            boxes = rois[sel, 1:]
            scores = cls_prob[sel].float()
            pred = clip_boxes(bbox_transform_inv(boxes, bbox_pred[sel].float()), float(im_info[b, 0]),
                              float(im_info[b, 1])) / float(im_info[b, 2])
            dets = []
            for c in range(self.n):
                if c == self.bg:
                    continue
                s = scores[:, c]
                m = s > self.thresh
                if not m.any():
                    continue
                bx = pred[m, 4 * c:4 * c + 4]
                keep = nms(bx, s[m], self.nms_thresh, bx.shape[0])
                dets.append(torch.cat([torch.full((keep.numel(), 1), float(c), device=bx.device), s[m][keep, None],
                                       bx[keep]], 1))
            d = torch.cat(dets) if dets else torch.zeros(0, 6, device=rois.device)
            if d.shape[0] > self.max_per_image:
                d = d[d[:, 1].argsort(descending=True)[:self.max_per_image]]
            out.append(d)
        return out


def _vgg16_conv5():
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512]
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2, ceil_mode=True))
        else:
            layers += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers), 512


class _CReLU(nn.Module):
    """PVANet concatenated ReLU: conv -> [x, -x] -> scale/shift -> ReLU."""

    def __init__(self, cin, cout, k, stride=1):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride, k // 2)
        self.bn = nn.BatchNorm2d(2 * cout)

    def forward(self, x):
        y = self.conv(x)
        return F.relu(self.bn(torch.cat([y, -y], 1)))


class _Inception(nn.Module):
    def __init__(self, cin, cout, stride=1):
        super().__init__()
        b = cout // 4
        self.b1 = nn.Sequential(nn.Conv2d(cin, b, 1, stride), nn.ReLU(True))
        self.b3 = nn.Sequential(nn.Conv2d(cin, b, 1), nn.ReLU(True), nn.Conv2d(b, b, 3, stride, 1), nn.ReLU(True))
        self.b5 = nn.Sequential(nn.Conv2d(cin, b, 1), nn.ReLU(True), nn.Conv2d(b, b, 3, 1, 1), nn.ReLU(True),
                                nn.Conv2d(b, b, 3, stride, 1), nn.ReLU(True))
        self.bp = nn.Sequential(nn.MaxPool2d(3, stride, 1), nn.Conv2d(cin, cout - 3 * b, 1), nn.ReLU(True))
        self.proj = nn.Conv2d(cin, cout, 1, stride) if (cin != cout or stride != 1) else None

    def forward(self, x):
        y = torch.cat([self.b1(x), self.b3(x), self.b5(x), self.bp(x)], 1)
        return y + (x if self.proj is None else self.proj(x))


class _PVANetLite(nn.Module):
    """PVANet-style feature extractor (C.ReLU stem, inception stages, hyper-feature
    concat of conv3/conv4/conv5 at stride 16 -> 512 channels). Architecture parity
    with the released PVANet is unpinned: the reference loads its weights and graph
    from a downloaded BigDL model file."""

    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(_CReLU(3, 16, 7, 2), nn.MaxPool2d(3, 2, 1))                 # /4, 32 ch
        self.c2 = nn.Sequential(_CReLU(32, 32, 3), _CReLU(64, 32, 3))                        # /4, 64
        self.c3 = nn.Sequential(_CReLU(64, 64, 3, 2), _CReLU(128, 64, 3))                    # /8, 128
        self.c4 = nn.Sequential(_Inception(128, 256, 2), _Inception(256, 256))               # /16, 256
        self.c5 = nn.Sequential(_Inception(256, 384, 2), _Inception(384, 384))               # /32, 384
        self.fuse = nn.Sequential(nn.Conv2d(128 + 256 + 384, 512, 1), nn.ReLU(True))

    def forward(self, x):
        x = self.c2(self.stem(x))
        c3 = self.c3(x)
        c4 = self.c4(c3)
        c5 = self.c5(c4)
        h, w = c4.shape[2], c4.shape[3]
        hyper = torch.cat([F.max_pool2d(c3, 3, 2, 1)[:, :, :h, :w], c4,
                           F.interpolate(c5, size=(h, w), mode="bilinear", align_corners=False)], 1)
        return self.fuse(hyper)


def _vgg_native(seq, x):
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.Conv2d):
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            x = _nconv(x, m, "relu" if relu else None)
            i += 2 if relu else 1
            continue
        if isinstance(m, nn.MaxPool2d):
            x = ops.max_pool2d_nhwc(x, (m.kernel_size, m.kernel_size), (m.stride, m.stride), (m.padding, m.padding),
                                    ceil_mode=m.ceil_mode)
        i += 1
    return x


def _crelu_native(u, x):
    y = _nconv(x, u.conv)
    z = torch.cat([y, -y], -1)
    bn = u.bn
    return ops.batch_norm_nhwc(z.contiguous(), bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps,
                               bn.momentum if bn.momentum is not None else 0.1, relu=True,
                               training=bn.training)


def _seq_native(seq, x):
    """nn.Sequential of Conv2d / ReLU / MaxPool2d on NHWC (inception branches)."""
    return _vgg_native(seq, x)


def _inception_native(u, x):
    ys = [_seq_native(u.b1, x), _seq_native(u.b3, x), _seq_native(u.b5, x), _seq_native(u.bp, x)]
    y = torch.cat(ys, -1)
    return y + (x if u.proj is None else _nconv(x, u.proj))


def _pvanet_native(net, x):
    from zoo.ops.layers import resize_bilinear
    x = _crelu_native(net.stem[0], x)
    x = ops.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))
    for u in net.c2:
        x = _crelu_native(u, x)
    c3 = x
    for u in net.c3:
        c3 = _crelu_native(u, c3)
    c4 = c3
    for u in net.c4:
        c4 = _inception_native(u, c4)
    c5 = c4
    for u in net.c5:
        c5 = _inception_native(u, c5)
    h, w = c4.shape[1], c4.shape[2]
    p3 = ops.max_pool2d_nhwc(c3, (3, 3), (2, 2), (1, 1))[:, :h, :w]
    hyper = torch.cat([p3, c4, resize_bilinear(c5.contiguous(), h, w, align=2)], -1)   # half-pixel
    return _nconv(hyper.contiguous(), net.fuse[0], "relu")


class FasterRCNN(nn.Module):
    """backbone (stride 16) -> RPN -> Proposal -> RoI pooling -> fc heads.
    forward(x, im_info) -> (rois [R, 5], cls_prob [R, C], bbox_pred [R, 4C])."""

    def __init__(self, num_classes=21, backbone="vgg16", pre_nms_topn=6000, post_nms_topn=300):
        super().__init__()
        self.num_classes = num_classes
        if backbone == "vgg16":
            self.features, c = _vgg16_conv5()
            fc_in, fc = 512 * 7 * 7, 4096
        elif backbone == "pvanet":
            self.features, c = _PVANetLite(), 512
            fc_in, fc = 512 * 6 * 6, 2048
        else:
            raise ValueError("backbone must be 'vgg16' or 'pvanet'")
        self.pooled = 7 if backbone == "vgg16" else 6
        A = 9
        self.rpn_conv = nn.Conv2d(c, 512 if backbone == "vgg16" else 384, 3, padding=1)
        rc = self.rpn_conv.out_channels
        self.rpn_cls = nn.Conv2d(rc, 2 * A, 1)
        self.rpn_bbox = nn.Conv2d(rc, 4 * A, 1)
        self.proposal = Proposal(pre_nms_topn, post_nms_topn)
        self.fc6 = nn.Linear(fc_in, fc)
        self.fc7 = nn.Linear(fc, fc)
        self.cls_score = nn.Linear(fc, num_classes)
        self.bbox_pred = nn.Linear(fc, 4 * num_classes)

    def features_nhwc(self, x):
        """GPU backbone: NCHW fp32 image -> NHWC bf16 stride-16 features (native kernels)."""
        xn = ops.native().nchw_to_nhwc(x.float().contiguous(), 4)        # 3 -> 4 channels, bf16
        if isinstance(self.features, nn.Sequential):
            return _vgg_native(self.features, xn)
        return _pvanet_native(self.features, xn)

    def _forward_native(self, x, im_info):
        f = self.features_nhwc(x)
        r = _nconv(f, self.rpn_conv, "relu")
        s = _nconv(r, self.rpn_cls)                                       # [B, H, W, 2A]
        B, H, W, twoA = s.shape
        A = twoA // 2
        from zoo.ops.nn import softmax
        prob = softmax(s.float().reshape(B, H, W, 2, A), dim=3).reshape(B, H, W, twoA)
        deltas = _nconv(r, self.rpn_bbox).float()
        rois = self.proposal(prob.permute(0, 3, 1, 2), deltas.permute(0, 3, 1, 2), im_info)
        pooled = roi_pool_nhwc(f, rois, self.pooled)                      # [R, P, P, C]
        pooled = pooled.permute(0, 3, 1, 2).flatten(1)                    # the fc6 weight's (C, P, P) order
        h = ops.linear(pooled, self.fc6.weight, self.fc6.bias, act="relu")
        h = ops.linear(h, self.fc7.weight, self.fc7.bias, act="relu")
        cls = softmax(ops.linear(h, self.cls_score.weight, self.cls_score.bias).float(), -1)
        box = ops.linear(h, self.bbox_pred.weight, self.bbox_pred.bias).float()
        return rois, cls, box

    def forward(self, x, im_info):
        if x.is_cuda:
            return self._forward_native(x, im_info)
        f = self.features(x)
        r = F.relu(self.rpn_conv(f))
        s = self.rpn_cls(r)
        B, twoA, H, W = s.shape
        prob = F.softmax(s.reshape(B, 2, twoA // 2, H, W), 1).reshape(B, twoA, H, W)
        rois = self.proposal(prob, self.rpn_bbox(r), im_info)
        pooled = roi_pool(f, rois, self.pooled).flatten(1)
        h = F.relu(ops.linear(pooled, self.fc6.weight, self.fc6.bias).float())
        h = F.relu(ops.linear(h, self.fc7.weight, self.fc7.bias).float())
        cls = F.softmax(ops.linear(h, self.cls_score.weight, self.cls_score.bias).float(), -1)
        box = ops.linear(h, self.bbox_pred.weight, self.bbox_pred.bias).float()
        return rois, cls, box


def aspect_scale(img_hwc, resolution=600, scale_multiple_of=1, max_size=1000):
    """ImageAspectScale(resolution, scaleMultipleOf) + ImageChannelNormalize(means) + ImInfo:
    HWC BGR image -> (CHW float32 array, im_info [h, w, scale])."""
    from zoo.feature.image.transforms import resize_bilinear
    h, w = img_hwc.shape[:2]
    scale = resolution / float(min(h, w))
    if round(scale * max(h, w)) > max_size:
        scale = max_size / float(max(h, w))
    nh, nw = int(round(h * scale)), int(round(w * scale))
    if scale_multiple_of > 1:
        nh = max(scale_multiple_of, nh // scale_multiple_of * scale_multiple_of)
        nw = max(scale_multiple_of, nw // scale_multiple_of * scale_multiple_of)
    out = resize_bilinear(img_hwc.astype(np.float32), nh, nw)
    out = out - np.asarray(FRCNN_MEANS, np.float32)
    return out.transpose(2, 0, 1).copy(), np.asarray([nh, nw, nh / float(h)], np.float32)
