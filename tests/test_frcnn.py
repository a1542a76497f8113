"""Faster R-CNN configs of ObjectDetector (M6) + detection post-processing
(Postprocessor.scala, LabelReader.scala) + the native NMS bitmask kernel (HK21).
Anchors are pinned against the published py-faster-rcnn generate_anchors table."""
import numpy as np
import pytest
import torch

from zoo.models.image.objectdetection import (DecodeOutput, DetectionOutputFrcnn, ObjectDetector, Proposal,
                                              ScaleDetection, Visualizer, generate_anchors, nms,
                                              read_pascal_label_map, roi_pool)
from zoo.models.image.objectdetection.frcnn import bbox_transform_inv


def test_anchors_match_reference_table():
    a = generate_anchors()
    ref = [[-84, -40, 99, 55], [-176, -88, 191, 103], [-360, -184, 375, 199], [-56, -56, 71, 71],
           [-120, -120, 135, 135], [-248, -248, 263, 263], [-36, -80, 51, 95], [-80, -168, 95, 183],
           [-168, -344, 183, 359]]
    assert a.tolist() == ref


def test_bbox_transform_zero_deltas_is_identity():
    boxes = torch.tensor([[10.0, 20.0, 50.0, 80.0], [0.0, 0.0, 15.0, 15.0]])
    out = bbox_transform_inv(boxes, torch.zeros(2, 8))
    torch.testing.assert_close(out[:, :4], boxes)
    torch.testing.assert_close(out[:, 4:], boxes)


def test_roi_pool_is_max_over_bins():
    f = torch.arange(2 * 3 * 8 * 8, dtype=torch.float32).reshape(2, 3, 8, 8)
    rois = torch.tensor([[1.0, 0.0, 0.0, 56.0, 56.0]])  # whole 8x8 map at scale 1/8 (round(56/8) = 7)
    out = roi_pool(f, rois, pooled=2, spatial_scale=1 / 8)
    exp = torch.nn.functional.adaptive_max_pool2d(f[1:2], 2)[0]
    torch.testing.assert_close(out[0], exp)
    # BigDL / Caffe bins: roi 0..8 (9 wide, past the map) -> bin 0 = [0, 5), bin 1 = [4, 9) clipped to 8
    out = roi_pool(f, torch.tensor([[0.0, 0.0, 0.0, 63.0, 63.0]]), pooled=2, spatial_scale=1 / 8)
    torch.testing.assert_close(out[0, :, 0, 0], f[0, :, :5, :5].amax((1, 2)))
    torch.testing.assert_close(out[0, :, 1, 1], f[0, :, 4:, 4:].amax((1, 2)))


def test_proposal_and_detection_output():
    torch.manual_seed(0)
    B, A, H, W = 1, 9, 6, 8
    prob = torch.rand(B, 2 * A, H, W)
    deltas = torch.randn(B, 4 * A, H, W) * 0.1
    info = torch.tensor([[96.0, 128.0, 1.0]])
    rois = Proposal(pre_nms_topn=100, post_nms_topn=10, min_size=4)(prob, deltas, info)
    assert rois.shape[1] == 5 and 0 < rois.shape[0] <= 10
    assert (rois[:, 1] >= 0).all() and (rois[:, 3] <= 127).all() and (rois[:, 4] <= 95).all()
    # detection output: one confident class-3 RoI survives, a duplicate is suppressed
    r = torch.tensor([[0, 10.0, 10.0, 40.0, 40.0], [0, 11.0, 11.0, 41.0, 41.0], [0, 60.0, 60.0, 90.0, 90.0]])
    cls = torch.full((3, 5), 0.01)
    cls[0, 3], cls[1, 3], cls[2, 1] = 0.9, 0.8, 0.7
    det = DetectionOutputFrcnn(num_classes=5)(r, cls, torch.zeros(3, 20), torch.tensor([[100.0, 100.0, 2.0]]))[0]
    labels = sorted(det[:, 0].tolist())
    assert labels == [1.0, 3.0]
    d3 = det[det[:, 0] == 3][0]
    torch.testing.assert_close(d3[2:], torch.tensor([5.0, 5.0, 20.0, 20.0]))  # divided by the scale 2


def test_frcnn_detector_configs_end_to_end():
    torch.manual_seed(0)
    for name in ("frcnn-vgg16", "frcnn-pvanet-quantize"):
        d = ObjectDetector(name, pre_nms_topn=200, post_nms_topn=16)
        assert type(d).__name__ == "FrcnnDetector"
        d.resolution = 96 if d.backbone == "vgg16" else 128
        d.detect.thresh = 0.0
        img = (np.random.rand(100, 140, 3) * 255).astype(np.uint8)
        out = d.detect_images([img])[0]
        assert out.ndim == 2 and out.shape[1] == 6 and 0 < out.shape[0] <= 100
        assert (out[:, 2] >= 0).all() and (out[:, 4] <= 140 + 1).all()


def test_postprocessors_and_label_maps():
    assert read_pascal_label_map()[15] == "person"
    flat = np.array([2, 1, 0.9, 0.1, 0.1, 0.5, 0.5, 3, 0.8, 0.2, 0.2, 0.4, 0.9], np.float32)
    d = DecodeOutput()(flat)
    assert d.shape == (2, 6)
    s = ScaleDetection()(d, (200, 100))
    np.testing.assert_allclose(s[0, 2:], [10, 20, 50, 100])
    img = Visualizer(thresh=0.5)(np.zeros((200, 100, 3), np.uint8), s)
    assert img.sum() > 0


def _rand_boxes(n, seed):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(n, 2, generator=g) * 100
    wh = torch.rand(n, 2, generator=g) * 30 + 2
    return torch.cat([xy, xy + wh], 1), torch.rand(n, generator=g)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 500, 3000])
def test_native_nms_matches_cpu(gpu, n):
    b, s = _rand_boxes(n, n)
    ref = nms(b, s, 0.5, n)
    got = nms(b.to(gpu), s.to(gpu), 0.5, n)
    assert got.cpu().tolist() == ref.tolist()
    got5 = nms(b.to(gpu), s.to(gpu), 0.5, n, max_keep=5)
    assert got5.cpu().tolist() == ref[:5].tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_native_roi_pool_matches_reference(gpu, dt):
    from zoo.models.image.objectdetection.frcnn import roi_pool_nhwc
    torch.manual_seed(0)
    f = torch.randn(2, 16, 24, 40)
    rois = torch.tensor([[0, 0, 0, 300, 200], [1, 40, 30, 120, 90], [1, -20, 5, 700, 400], [0, 64, 64, 64, 64],
                         [1, 100.4, 20.6, 180.2, 150.9]], dtype=torch.float32)
    ref = roi_pool(f.to(dt).float(), rois, pooled=7, spatial_scale=1 / 16)
    fn = f.to(dt).permute(0, 2, 3, 1).contiguous().to(gpu).requires_grad_(True)
    out = roi_pool_nhwc(fn, rois.to(gpu), 7, 1 / 16)
    torch.testing.assert_close(out.float().permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=0)
    # backward: gradient routed to each bin's first argmax (Caffe), summed where RoIs overlap
    # (bf16 features tie often, so autograd through amax -- which splits between ties -- is not
    # the reference)
    _, arg = roi_pool(f.to(dt).float(), rois, pooled=7, spatial_scale=1 / 16, return_argmax=True)
    dy = torch.randn(5, 16, 7, 7)
    ref_g = torch.zeros(2, 16, 24 * 40)
    bidx = rois[:, 0].long()
    for i in range(rois.shape[0]):
        a = arg[i].reshape(16, -1)
        d = dy[i].reshape(16, -1).to(dt).float()
        ok = a >= 0
        ref_g[bidx[i]].scatter_add_(1, a.clamp_min(0), torch.where(ok, d, torch.zeros_like(d)))
    out.backward(dy.permute(0, 2, 3, 1).to(gpu).to(out.dtype))
    torch.testing.assert_close(fn.grad.float().permute(0, 3, 1, 2).cpu(), ref_g.reshape(2, 16, 24, 40),
                               rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("backbone", ["vgg16", "pvanet"])
def test_frcnn_native_backbone_and_heads(gpu, backbone):
    """The GPU path (native NHWC convs, pools, C.ReLU BN, resize, RoI pool, fc heads) against
    the fp32 torch reference of the same weights; no MIOpen / hipBLASLt kernel runs."""
    from torch.profiler import ProfilerActivity, profile
    from zoo.models.image.objectdetection.frcnn import FasterRCNN
    torch.manual_seed(0)
    m = FasterRCNN(num_classes=21, backbone=backbone, pre_nms_topn=600, post_nms_topn=50).eval()
    for mod in m.modules():       # keep activations O(1) through the deep stack
        if isinstance(mod, torch.nn.Conv2d):
            torch.nn.init.normal_(mod.weight, 0, (2.0 / (mod.in_channels * mod.kernel_size[0] ** 2)) ** 0.5)
    x = torch.randn(1, 3, 224, 320)
    with torch.no_grad():
        ref = m.features(x)
        g = m.to(gpu)
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            f = g.features_nhwc(x.to(gpu))
            rois, cls, box = g(x.to(gpu), torch.tensor([[224.0, 320.0, 1.0]], device=gpu))
            torch.cuda.synchronize()
    out = f.float().permute(0, 3, 1, 2).cpu()
    assert out.shape == ref.shape
    assert ((out - ref).norm() / ref.norm()).item() < 3e-2
    assert rois.shape[1] == 5 and cls.shape == (rois.shape[0], 21) and box.shape == (rois.shape[0], 84)
    assert torch.allclose(cls.sum(-1), torch.ones_like(cls.sum(-1)), atol=1e-3)
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    bad = sorted({n for n in names if any(b in n for b in ("MIOpen", "miopen", "naive_conv", "Cijk_"))})
    assert not bad, bad[:5]
    assert any("roi_pool" in n for n in names)


@pytest.mark.gpu
def test_frcnn_on_gpu(gpu):
    torch.manual_seed(0)
    d = ObjectDetector("frcnn-vgg16", pre_nms_topn=2000, post_nms_topn=100).to(gpu)
    d.resolution = 224
    d.detect.thresh = 0.0
    out = d.detect_images([(np.random.rand(200, 300, 3) * 255).astype(np.uint8)])[0]
    assert out.shape[1] == 6 and 0 < out.shape[0] <= 100


def test_ssd_mobilenet_config_shapes():
    from zoo.models.image.objectdetection import SSDMobileNet
    d = ObjectDetector("ssd-mobilenet-300x300")
    assert isinstance(d.ssd, SSDMobileNet)
    loc, conf = d.ssd(torch.randn(1, 3, 300, 300))
    P = d.ssd.priors.shape[0]
    assert loc.shape == (1, P, 4) and conf.shape == (1, P, 21)
    assert P == 19 * 19 * 4 + (100 + 25 + 9 + 4 + 1) * 6
    dets = d.detect_batch(np.random.rand(1, 3, 300, 300).astype(np.float32))
    assert dets[0].shape[1] == 6


def test_half_pixel_resize_reference_matches_interpolate():
    """resize mode 2 (PVANet hyper-feature upsampling on the GPU path) is PyTorch's
    align_corners=False bilinear: the NHWC reference agrees with F.interpolate."""
    import torch.nn.functional as F
    from zoo.ops.layers import resize_bilinear_ref
    torch.manual_seed(0)
    x = torch.randn(2, 5, 7, 3)
    for oh, ow in [(10, 14), (9, 4), (5, 7)]:
        ref = F.interpolate(x.permute(0, 3, 1, 2), size=(oh, ow), mode="bilinear", align_corners=False)
        out = resize_bilinear_ref(x, oh, ow, align=2).permute(0, 3, 1, 2)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
