"""SSD object detection (Zs/models/image/objectdetection/ssd/SSD.scala:35-214, SSDGraph.scala:28-220;
common/nn/PriorBox, NormalizeScale, DetectionOutputSSD; common/loss/MultiBoxLoss.scala;
common/BboxUtil.scala; common/evaluation/MeanAveragePrecision.scala; Py objectdetection/).

Boxes are (x1, y1, x2, y2) normalised to [0, 1]. Priors are SSD "center-size"
boxes; offsets are encoded with variances (0.1, 0.1, 0.2, 0.2). NMS runs on
the device (vectorised IoU matrix + greedy suppression per class).
"""
import itertools
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo.models.image.imageclassification.image_classifier import ImageModel


# ---- box utilities (BboxUtil) ------------------------------------------------------------------
def iou_matrix(a, b):
    """a [N, 4], b [M, 4] (x1, y1, x2, y2) -> IoU [N, M]."""
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    area_a = ((a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]))[:, None]
    area_b = ((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]))[None, :]
    return inter / (area_a + area_b - inter).clamp(min=1e-12)


def center_to_corner(p):
    return torch.cat([p[..., :2] - p[..., 2:] / 2, p[..., :2] + p[..., 2:] / 2], -1)


def corner_to_center(b):
    return torch.cat([(b[..., :2] + b[..., 2:]) / 2, b[..., 2:] - b[..., :2]], -1)


def encode(gt, priors, var=(0.1, 0.1, 0.2, 0.2)):
    """gt corners [P, 4], priors center-size [P, 4] -> regression targets [P, 4]."""
    g = corner_to_center(gt)
    d_xy = (g[:, :2] - priors[:, :2]) / (priors[:, 2:] * var[0])
    d_wh = torch.log(g[:, 2:].clamp(min=1e-12) / priors[:, 2:]) / var[2]
    return torch.cat([d_xy, d_wh], 1)


def decode(loc, priors, var=(0.1, 0.1, 0.2, 0.2)):
    if loc.is_cuda and loc.dim() == 3 and priors.dim() == 2 and var[0] == var[1] and var[2] == var[3]:
        from zoo.ops.pointwise import box_decode   # native decode kernel (HK21)
        return box_decode(loc, priors, (var[0], var[2]))
    xy = priors[..., :2] + loc[..., :2] * var[0] * priors[..., 2:]
    wh = priors[..., 2:] * torch.exp(loc[..., 2:] * var[2])
    return center_to_corner(torch.cat([xy, wh], -1))


def nms(boxes, scores, iou_threshold=0.45, top_k=400, max_keep=0):
    """Greedy NMS; returns kept indices (descending score). On the GPU the IoU
    suppression bitmask comes from the native kernel (csrc/kernels/detect.hip)."""
    order = scores.argsort(descending=True)[:top_k]
    if order.numel() == 0:
        return order
    if boxes.is_cuda:
        from zoo.ops._native import native
        k = native().nms_sorted(boxes[order].float().contiguous(), float(iou_threshold), int(max_keep))
        return order[k]
    b = boxes[order]
    iou = iou_matrix(b, b)
    n = order.numel()
    keep = torch.ones(n, dtype=torch.bool, device=boxes.device)
    iou_cpu = iou.cpu()
    kc = keep.cpu()
    for i in range(n):
        if kc[i]:
            kc[i + 1:] &= iou_cpu[i, i + 1:] <= iou_threshold
    return order[kc.to(boxes.device)]


# ---- priors (PriorBox) ---------------------------------------------------------------------------
class SSDConfig:
    def __init__(self, resolution=300, feature_maps=(38, 19, 10, 5, 3, 1), steps=(8, 16, 32, 64, 100, 300),
                 min_sizes=(30, 60, 111, 162, 213, 264), max_sizes=(60, 111, 162, 213, 264, 315),
                 aspect_ratios=((2,), (2, 3), (2, 3), (2, 3), (2,), (2,)), clip=True,
                 variances=(0.1, 0.1, 0.2, 0.2)):
        self.resolution, self.feature_maps, self.steps = resolution, feature_maps, steps
        self.min_sizes, self.max_sizes, self.aspect_ratios = min_sizes, max_sizes, aspect_ratios
        self.clip, self.variances = clip, variances

    def boxes_per_location(self):
        return [2 + 2 * len(a) for a in self.aspect_ratios]


def prior_boxes(cfg):
    """All priors, center-size normalised [P, 4], in head order (map, y, x, box)."""
    out = []
    for k, f in enumerate(cfg.feature_maps):
        for i, j in itertools.product(range(f), repeat=2):
            fk = cfg.resolution / cfg.steps[k]
            cx, cy = (j + 0.5) / fk, (i + 0.5) / fk
            s = cfg.min_sizes[k] / cfg.resolution
            out.append([cx, cy, s, s])
            sp = math.sqrt(s * (cfg.max_sizes[k] / cfg.resolution))
            out.append([cx, cy, sp, sp])
            for ar in cfg.aspect_ratios[k]:
                r = math.sqrt(ar)
                out.append([cx, cy, s * r, s / r])
                out.append([cx, cy, s / r, s * r])
    p = torch.tensor(out, dtype=torch.float32)
    return p.clamp(0, 1) if cfg.clip else p


class NormalizeScale(nn.Module):
    """Channel-wise L2 normalisation with a learnable per-channel scale (init 20);
    channels last (NHWC)."""

    def __init__(self, channels, scale=20.0, eps=1e-10):
        super().__init__()
        self.weight = nn.Parameter(torch.full((channels,), float(scale)))
        self.eps = eps

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
            return _L2NormScaleFn.apply(x.contiguous(), self.weight, float(self.eps))
        xf = x.float()
        n = xf.pow(2).sum(-1, keepdim=True).sqrt() + self.eps
        return (xf / n * self.weight).to(x.dtype)


class _L2NormScaleFn(torch.autograd.Function):
    """One fused native pass each way (csrc/kernels/detect.hip l2norm_scale_*): the torch
    composition re-read the [B, 38, 38, 512] map five times forward and eight backward."""

    @staticmethod
    def forward(ctx, x, w, eps):
        from zoo.ops._native import native
        y, n = native().l2norm_scale_fwd(x, w.float().contiguous(), eps)
        ctx.save_for_backward(x, w, n)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, g):
        from zoo.ops._native import native
        x, w, n = ctx.saved_tensors
        dx, dw = native().l2norm_scale_bwd(g.contiguous().to(x.dtype), x, w.float().contiguous(), n, ctx.eps)
        return dx, dw.to(w.dtype), None


def mine_hard_negatives(ce, pos, ratio):
    """pos | the ceil(ratio * #pos) (<= P - 1) highest-loss negatives of each row, ties taken in
    prior order (MultiBoxLoss.scala hard negative mining). ce [B, P] per-prior loss."""
    B, P = ce.shape
    if ce.is_cuda:
        from zoo.ops._native import native
        conf = pos.long() if pos.dtype == torch.bool else pos
        # the kernel takes labels; any label != bg (0 here) marks a positive
        return native().ssd_mine(ce.detach().float().contiguous(), conf.contiguous(), 0, float(ratio)).bool()
    neg_ce = ce.detach().float().masked_fill(pos, 0).clamp_min(0)
    order = torch.sort(neg_ce, dim=1, descending=True, stable=True).indices
    rank = torch.empty_like(order)
    rank.scatter_(1, order, torch.arange(P, device=ce.device).expand(B, P))
    k = torch.ceil(float(ratio) * pos.sum(1, keepdim=True).float()).clamp(max=P - 1)
    return pos | (rank < k)


def _vgg16_base():
    """SSD's VGG16 trunk on the native NHWC units (conv4_3 is index 12: its ReLU output
    feeds the L2-normalised head; fc6 is the dilated 3x3, fc7 the 1x1)."""
    from zoo.models.image.native_nets import CB, MaxPool
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "C", 512, 512, 512, "M", 512, 512, 512]
    layers, c = [], 4
    for v in cfg:
        if v == "M":
            layers.append(MaxPool(2, 2))
        elif v == "C":
            layers.append(MaxPool(2, 2, ceil_mode=True))
        else:
            layers.append(CB(c, v, 3, 1, 1))
            c = v
    layers += [MaxPool(3, 1, 1), CB(512, 1024, 3, 1, 6, dil=6), CB(1024, 1024, 1)]
    return nn.ModuleList(layers)


def _heads(chans, nb, num_classes):
    from zoo.models.image.native_nets import CB
    loc = nn.ModuleList([CB(c, n * 4, 3, 1, 1, relu=False) for c, n in zip(chans, nb)])
    conf = nn.ModuleList([CB(c, n * num_classes, 3, 1, 1, relu=False) for c, n in zip(chans, nb)])
    return loc, conf


def _multibox(loc_heads, conf_heads, feats, num_classes):
    """NHWC head outputs [B, H, W, n*4] flatten straight into [B, H*W*n, 4]."""
    B = feats[0].shape[0]
    loc = torch.cat([l(f).reshape(B, -1, 4) for l, f in zip(loc_heads, feats)], 1).float()
    conf = torch.cat([c(f).reshape(B, -1, num_classes) for c, f in zip(conf_heads, feats)], 1).float()
    return loc, conf


class SSD(nn.Module):
    """SSD-VGG16 (300x300 by default) on the native NHWC bf16 conv kernels.
    forward(NCHW images) -> (loc [B, P, 4], conf [B, P, C]) in fp32."""

    def __init__(self, num_classes=21, cfg=None):
        super().__init__()
        from zoo.models.image.native_nets import CB
        self.cfg = cfg or SSDConfig()
        self.num_classes = num_classes
        self.base = _vgg16_base()
        self.l2norm = NormalizeScale(512, 20.0)
        self.extras = nn.ModuleList([
            nn.Sequential(CB(1024, 256, 1), CB(256, 512, 3, 2, 1)),
            nn.Sequential(CB(512, 128, 1), CB(128, 256, 3, 2, 1)),
            nn.Sequential(CB(256, 128, 1), CB(128, 256, 3)),
            nn.Sequential(CB(256, 128, 1), CB(128, 256, 3))])
        chans = [512, 1024, 512, 256, 256, 256]
        self.loc, self.conf = _heads(chans, self.cfg.boxes_per_location(), num_classes)
        self.register_buffer("priors", prior_boxes(self.cfg))

    def forward(self, x):
        from zoo.models.image.native_nets import to_nhwc
        x = to_nhwc(x, 3, 4)
        feats = []
        for i, l in enumerate(self.base):
            x = l(x)
            if i == 12:  # conv4_3 (+ReLU)
                feats.append(self.l2norm(x))
        feats.append(x)
        for e in self.extras:
            x = e(x)
            feats.append(x)
        return _multibox(self.loc, self.conf, feats, self.num_classes)


class SSDMobileNet(nn.Module):
    """SSD-MobileNet-300 ("ssd-mobilenet-300x300", ObjectDetectionConfig.scala:64-69): MobileNet v1
    taps at conv11 (19x19, 512) and conv13 (10x10, 1024) plus four extra 1x1/3x3-s2
    stages, all on the native NHWC units. forward -> (loc [B, P, 4], conf [B, P, C])."""

    CONFIG = dict(resolution=300, feature_maps=(19, 10, 5, 3, 2, 1), steps=(16, 32, 64, 100, 150, 300),
                  min_sizes=(60, 105, 150, 195, 240, 285), max_sizes=(105, 150, 195, 240, 285, 300),
                  aspect_ratios=((2,), (2, 3), (2, 3), (2, 3), (2, 3), (2, 3)))

    def __init__(self, num_classes=21):
        super().__init__()
        from zoo.models.image.native_nets import CB, MobileNet
        self.cfg = SSDConfig(**self.CONFIG)
        self.num_classes = num_classes
        self.base = MobileNet(1000).features          # classifier head dropped
        self.tap = 22                                 # conv11 pointwise output (stride 16)

        def extra(cin, mid, cout):
            return nn.Sequential(CB(cin, mid, 1), CB(mid, cout, 3, 2, 1))
        self.extras = nn.ModuleList([extra(1024, 256, 512), extra(512, 128, 256), extra(256, 128, 256),
                                     extra(256, 64, 128)])
        chans = [512, 1024, 512, 256, 256, 128]
        self.loc, self.conf = _heads(chans, self.cfg.boxes_per_location(), num_classes)
        self.register_buffer("priors", prior_boxes(self.cfg))

    def forward(self, x):
        from zoo.models.image.native_nets import to_nhwc
        x = to_nhwc(x, 3, 4)
        feats = []
        for i, l in enumerate(self.base):
            x = l(x)
            if i == self.tap:
                feats.append(x)
        feats.append(x)
        for e in self.extras:
            x = e(x)
            feats.append(x)
        return _multibox(self.loc, self.conf, feats, self.num_classes)


class DetectionOutputSSD(nn.Module):
    """Decode + per-class threshold + NMS + keep_top_k -> list of [K, 6] (label, score, x1, y1, x2, y2)."""

    def __init__(self, num_classes=21, bg_label=0, nms_thresh=0.45, nms_topk=400, keep_topk=200,
                 conf_thresh=0.01, variances=(0.1, 0.1, 0.2, 0.2)):
        super().__init__()
        self.n, self.bg, self.nms_thresh, self.nms_topk = num_classes, bg_label, nms_thresh, nms_topk
        self.keep_topk, self.conf_thresh, self.var = keep_topk, conf_thresh, variances

    @torch.no_grad()
    def forward(self, loc, conf, priors):
        boxes = decode(loc, priors, self.var).clamp(0, 1)
        scores = F.softmax(conf.float(), -1)
        out = []
        for b in range(loc.shape[0]):
            dets = []
            for c in range(self.n):
                if c == self.bg:
                    continue
                s = scores[b, :, c]
                m = s > self.conf_thresh
                if not m.any():
                    continue
                bx, sc = boxes[b][m], s[m]
                keep = nms(bx, sc, self.nms_thresh, self.nms_topk)
                lab = torch.full((keep.numel(), 1), float(c), device=bx.device)
                dets.append(torch.cat([lab, sc[keep, None], bx[keep]], 1))
            d = torch.cat(dets) if dets else torch.zeros(0, 6, device=loc.device)
            if d.shape[0] > self.keep_topk:
                d = d[d[:, 1].argsort(descending=True)[:self.keep_topk]]
            out.append(d)
        return out


class MultiBoxLoss(nn.Module):
    """Matching (best prior per GT + IoU >= overlap), smooth-L1 on positives,
    softmax CE with 3:1 hard negative mining, normalised by #positives (MultiBoxLoss.scala)."""

    def __init__(self, num_classes=21, overlap=0.5, neg_pos_ratio=3.0, variances=(0.1, 0.1, 0.2, 0.2), bg_label=0):
        super().__init__()
        self.n, self.overlap, self.ratio, self.var, self.bg = num_classes, overlap, neg_pos_ratio, variances, bg_label

    def match(self, gt_boxes, gt_labels, priors):
        P = priors.shape[0]
        if gt_boxes.numel() == 0:
            return torch.zeros(P, 4, device=priors.device), torch.full((P,), self.bg, dtype=torch.long,
                                                                        device=priors.device)
        iou = iou_matrix(gt_boxes, center_to_corner(priors))        # [G, P]
        best_gt_iou, best_gt = iou.max(0)
        best_prior = iou.argmax(1)
        best_gt_iou[best_prior] = 2.0
        best_gt[best_prior] = torch.arange(gt_boxes.shape[0], device=priors.device)
        labels = gt_labels[best_gt].long().clone()
        labels[best_gt_iou < self.overlap] = self.bg
        return encode(gt_boxes[best_gt], priors, self.var), labels

    def match_native(self, targets, priors):
        """All images at once on the GPU (csrc/kernels/detect.hip ssd_match, HK21)."""
        from zoo.ops._native import native
        dev = priors.device
        G = max([int(t.shape[0]) for t in targets] + [1])
        gt = torch.zeros(len(targets), G, 5, device=dev)
        for i, t in enumerate(targets):
            if t.shape[0]:
                gt[i, :t.shape[0]] = t.to(dev).float()
        count = torch.tensor([int(t.shape[0]) for t in targets], dtype=torch.int32, device=dev)
        return native().ssd_match(gt, count, priors.float().contiguous(), float(self.overlap), float(self.var[0]),
                                  float(self.var[2]), int(self.bg))

    def forward(self, loc, conf, priors, targets):
        """targets: list of [G, 5] (label, x1, y1, x2, y2) per image."""
        B, P, _ = loc.shape
        if loc.is_cuda and self.var[0] == self.var[1] and self.var[2] == self.var[3]:
            loc_t, conf_t = self.match_native(targets, priors.to(loc.device))
        else:
            loc_t, conf_t = [], []
            for t in targets:
                t = t.to(loc.device)
                l, c = self.match(t[:, 1:], t[:, 0], priors)
                loc_t.append(l)
                conf_t.append(c)
            loc_t, conf_t = torch.stack(loc_t), torch.stack(conf_t)
        pos = conf_t != self.bg
        n_pos = pos.sum().clamp(min=1).float()
        # masked sums instead of boolean indexing: no nonzero / gather / index_put round trips
        sl1 = F.smooth_l1_loss(loc.float(), loc_t, reduction="none").sum(-1)
        loss_l = torch.where(pos, sl1, 0.0).sum()     # where, not *: a degenerate box's inf stays out
        ce = F.cross_entropy(conf.reshape(-1, self.n).float(), conf_t.reshape(-1), reduction="none").reshape(B, P)
        sel = mine_hard_negatives(ce, pos, self.ratio)
        loss_c = torch.where(sel, ce, 0.0).sum()
        return (loss_l + loss_c) / n_pos


# ---- evaluation (MeanAveragePrecision, VOC) ----------------------------------------------------------
def average_precision(recall, precision, use_07=True):
    if use_07:
        return float(np.mean([precision[recall >= t].max() if (recall >= t).any() else 0.0
                              for t in np.arange(0, 1.1, 0.1)]))
    mrec = np.concatenate([[0.0], recall, [1.0]])
    mpre = np.concatenate([[0.0], precision, [0.0]])
    for i in range(len(mpre) - 2, -1, -1):
        mpre[i] = max(mpre[i], mpre[i + 1])
    idx = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[idx + 1] - mrec[idx]) * mpre[idx + 1]))


def mean_average_precision(detections, ground_truths, num_classes, iou_thresh=0.5, use_07=True, bg_label=0):
    """detections: per image [K, 6] (label, score, box); ground_truths: per image [G, 5] (label, box)."""
    aps = []
    for c in range(num_classes):
        if c == bg_label:
            continue
        recs, n_gt = [], 0
        for img, (d, g) in enumerate(zip(detections, ground_truths)):
            g = np.asarray(g)
            gc = g[g[:, 0] == c][:, 1:] if len(g) else np.zeros((0, 4))
            n_gt += len(gc)
            d = np.asarray(d)
            for row in (d[d[:, 0] == c] if len(d) else []):
                recs.append((row[1], img, row[2:]))
        if n_gt == 0:
            continue
        recs.sort(key=lambda r: -r[0])
        used = {}
        tp = np.zeros(len(recs))
        for k, (_, img, box) in enumerate(recs):
            g = np.asarray(ground_truths[img])
            gc = g[g[:, 0] == c][:, 1:] if len(g) else np.zeros((0, 4))
            if len(gc):
                ious = iou_matrix(torch.tensor(box[None], dtype=torch.float32),
                                  torch.tensor(gc, dtype=torch.float32)).numpy()[0]
                j = int(ious.argmax())
                if ious[j] >= iou_thresh and not used.get((img, j)):
                    used[(img, j)] = True
                    tp[k] = 1
        ctp = np.cumsum(tp)
        recall = ctp / n_gt
        precision = ctp / np.arange(1, len(recs) + 1)
        aps.append(average_precision(recall, precision, use_07) if len(recs) else 0.0)
    return float(np.mean(aps)) if aps else 0.0


class ObjectDetector(ImageModel):
    """ObjectDetector facade: SSD-VGG16 (300/512) with DetectionOutputSSD, or a
    Faster R-CNN config ("frcnn-vgg16", "frcnn-pvanet") -> :class:`FrcnnDetector`."""

    def __new__(cls, model_name="ssd-vgg16-300x300", *a, **kw):
        if cls is ObjectDetector and str(model_name).startswith("frcnn"):
            return FrcnnDetector(model_name, *a, **kw)
        return super().__new__(cls)

    def __init__(self, model_name="ssd-vgg16-300x300", num_classes=21, label_map=None, **kwargs):
        super().__init__(**kwargs)
        res = 512 if "512" in model_name else 300
        cfg = SSDConfig() if res == 300 else SSDConfig(
            512, (64, 32, 16, 8, 4, 2, 1)[:6], (8, 16, 32, 64, 128, 256), (35.84, 76.8, 153.6, 230.4, 307.2, 384.0),
            (76.8, 153.6, 230.4, 307.2, 384.0, 460.8))
        self.model_name, self.num_classes, self.label_map = model_name, num_classes, label_map
        self.ssd = SSDMobileNet(num_classes) if "mobilenet" in model_name else SSD(num_classes, cfg)
        self.detect = DetectionOutputSSD(num_classes)
        self.criterion = MultiBoxLoss(num_classes)
        self.built = True

    def forward(self, x, *rest):
        return self.ssd(x)

    def _layer_list(self):
        return []

    @torch.no_grad()
    def detect_batch(self, x):
        was = self.training
        self.eval()
        dev = self.ssd.priors.device
        loc, conf = self.ssd(torch.as_tensor(x, dtype=torch.float32, device=dev))
        out = self.detect(loc, conf, self.ssd.priors)
        self.train(was)
        return [o.cpu().numpy() for o in out]


class FrcnnDetector(ImageModel):
    """Faster R-CNN ObjectDetector configs (ObjectDetectionConfig.scala:70-135):
    "frcnn-vgg16[-...]" (short side 600) and "frcnn-pvanet[-...]" (640, multiples of 32)."""

    def __init__(self, model_name="frcnn-vgg16", num_classes=21, label_map=None, pre_nms_topn=6000,
                 post_nms_topn=300, **kwargs):
        super().__init__(**kwargs)
        from zoo.models.image.objectdetection.frcnn import DetectionOutputFrcnn, FasterRCNN
        self.model_name, self.num_classes, self.label_map = model_name, num_classes, label_map
        self.backbone = "pvanet" if "pvanet" in model_name else "vgg16"
        self.resolution, self.multiple = (640, 32) if self.backbone == "pvanet" else (600, 1)
        self.frcnn = FasterRCNN(num_classes, self.backbone, pre_nms_topn, post_nms_topn)
        self.detect = DetectionOutputFrcnn(num_classes)
        self.built = True

    def forward(self, x, im_info):
        return self.frcnn(x, im_info)

    def _layer_list(self):
        return []

    @torch.no_grad()
    def detect_images(self, images_hwc_bgr):
        """Raw HWC BGR images (any sizes) -> per-image [K, 6] detections in original pixels."""
        from zoo.models.image.objectdetection.frcnn import aspect_scale
        was = self.training
        self.eval()
        dev = next(self.frcnn.parameters()).device
        out = []
        for img in images_hwc_bgr:
            chw, info = aspect_scale(np.asarray(img), self.resolution, self.multiple)
            x = torch.from_numpy(chw)[None].to(dev)
            ii = torch.from_numpy(info)[None].to(dev)
            rois, cls, box = self.frcnn(x, ii)
            out.append(self.detect(rois, cls, box, ii)[0].cpu().numpy())
        self.train(was)
        return out
