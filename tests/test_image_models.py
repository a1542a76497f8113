"""ImageClassifier configs and SSD object detection (ImageClassifierSpec,
SSDSpec / MultiBoxLossSpec / DetectionOutputSSDSpec / MeanAveragePrecisionSpec analogues)."""
import numpy as np
import pytest
import torch

from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


@pytest.mark.parametrize("name", ["squeezenet", "mobilenet", "mobilenet-v2", "alexnet", "inception-v1"])
def test_classifier_backbones_forward(name):
    from zoo.models.image.imageclassification import ImageClassifier
    m = ImageClassifier(name, num_classes=7).eval()
    size = 227 if name in ("alexnet", "squeezenet") else 224
    with torch.no_grad():
        out = m(torch.randn(2, 3, size, size))
    assert out.shape == (2, 7)


def test_predict_image_set_and_save_load(tmp_path):
    from zoo.feature.image import ImageSet
    from zoo.models.image.imageclassification import ImageClassifier
    torch.manual_seed(0)
    m = ImageClassifier("mobilenet", num_classes=5, label_map={0: "a", 1: "b", 2: "c", 3: "d", 4: "e"})
    imgs = [np.random.default_rng(i).integers(0, 255, (240 + 10 * i, 300, 3)).astype(np.uint8) for i in range(3)]
    res = m.predict_image_set(ImageSet.from_arrays(imgs))
    preds = [f["predict"] for f in res.features]
    assert all(len(p) == 5 and p[0][0] in "abcde" for p in preds)
    assert all(abs(sum(q for _, q in p) - 1.0) < 1e-4 for p in preds)
    m.save_model(str(tmp_path / "m.zoo"), over_write=True)
    m2 = ImageClassifier.load_model(str(tmp_path / "m.zoo"))
    x = torch.randn(1, 3, 224, 224)
    m.eval()
    m2.eval()
    with torch.no_grad():
        assert torch.allclose(m(x), m2(x), atol=1e-5)


def test_box_codec_and_iou():
    from zoo.models.image.objectdetection import decode, encode, iou_matrix
    pri = torch.tensor([[0.5, 0.5, 0.2, 0.3], [0.2, 0.3, 0.1, 0.1]])
    gt = torch.tensor([[0.35, 0.4, 0.62, 0.7], [0.1, 0.2, 0.3, 0.35]])
    assert torch.allclose(decode(encode(gt, pri), pri), gt, atol=1e-6)
    iou = iou_matrix(gt, gt)
    assert torch.allclose(iou.diag(), torch.ones(2)) and float(iou[0, 1]) == 0.0
    a = torch.tensor([[0.0, 0.0, 2.0, 2.0]])
    b = torch.tensor([[1.0, 1.0, 3.0, 3.0]])
    assert float(iou_matrix(a, b)) == pytest.approx(1 / 7)


def test_priors_and_ssd300_shapes():
    from zoo.models.image.objectdetection import SSD, SSDConfig, prior_boxes
    p = prior_boxes(SSDConfig())
    assert p.shape == (8732, 4) and float(p.min()) >= 0 and float(p.max()) <= 1
    ssd = SSD(num_classes=4).eval()
    with torch.no_grad():
        loc, conf = ssd(torch.randn(1, 3, 300, 300))
    assert loc.shape == (1, 8732, 4) and conf.shape == (1, 8732, 4)


def test_nms_and_detection_output():
    from zoo.models.image.objectdetection import DetectionOutputSSD, encode, nms
    boxes = torch.tensor([[0.1, 0.1, 0.5, 0.5], [0.12, 0.1, 0.5, 0.52], [0.6, 0.6, 0.9, 0.9]])
    keep = nms(boxes, torch.tensor([0.9, 0.8, 0.7]), 0.45)
    assert keep.tolist() == [0, 2]
    priors = torch.tensor([[0.3, 0.3, 0.4, 0.4], [0.31, 0.31, 0.4, 0.42], [0.75, 0.75, 0.3, 0.3]])
    loc = encode(boxes, priors)[None]
    conf = torch.tensor([[[0.0, 5.0, 0.0], [0.0, 4.0, 0.0], [0.0, 0.0, 6.0]]])
    det = DetectionOutputSSD(num_classes=3, conf_thresh=0.5)(loc, conf, priors)[0]
    labels = sorted(det[:, 0].tolist())
    assert labels == [1.0, 2.0]
    assert torch.allclose(det[det[:, 0] == 2][0, 2:], boxes[2], atol=1e-5)


def test_multibox_loss_decreases_when_fitting():
    from zoo.models.image.objectdetection import SSD, MultiBoxLoss, SSDConfig
    torch.manual_seed(0)
    cfg = SSDConfig()
    ssd = SSD(num_classes=3, cfg=cfg)
    crit = MultiBoxLoss(num_classes=3)
    x = torch.randn(2, 3, 300, 300)
    targets = [torch.tensor([[1.0, 0.1, 0.1, 0.4, 0.5]]), torch.tensor([[2.0, 0.5, 0.5, 0.9, 0.8],
                                                                        [1.0, 0.05, 0.6, 0.3, 0.95]])]
    opt = torch.optim.SGD(ssd.parameters(), lr=1e-3, momentum=0.9)
    losses = []
    for _ in range(4):
        loc, conf = ssd(x)
        loss = crit(loc, conf, ssd.priors, targets)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert np.isfinite(losses).all() and losses[-1] < losses[0]


def test_mean_average_precision():
    from zoo.models.image.objectdetection import mean_average_precision
    gts = [np.array([[1, 0.1, 0.1, 0.4, 0.4], [2, 0.5, 0.5, 0.9, 0.9]]), np.array([[1, 0.2, 0.2, 0.6, 0.6]])]
    perfect = [np.array([[1, 0.9, 0.1, 0.1, 0.4, 0.4], [2, 0.8, 0.5, 0.5, 0.9, 0.9]]),
               np.array([[1, 0.7, 0.2, 0.2, 0.6, 0.6]])]
    assert mean_average_precision(perfect, gts, 3) == pytest.approx(1.0)
    half = [np.array([[1, 0.9, 0.1, 0.1, 0.4, 0.4]]), np.zeros((0, 6))]
    m = mean_average_precision(half, gts, 3, use_07=False)
    assert 0 < m < 1


def test_hard_negative_mining_matches_rank_rule():
    """mine_hard_negatives == the reference's rank < ratio * #pos rule (distinct losses) and
    takes exactly ceil(ratio * #pos) negatives, clamped to P - 1."""
    import torch
    from zoo.models.image.objectdetection.ssd import mine_hard_negatives
    torch.manual_seed(0)
    B, P = 4, 200
    ce = torch.rand(B, P)
    pos = torch.rand(B, P) < 0.05
    pos[3] = torch.rand(P) < 0.5                      # 3 * #pos > P - 1: clamped
    sel = mine_hard_negatives(ce, pos, 3.0)
    neg_ce = ce.clone()
    neg_ce[pos] = 0
    rank = neg_ce.argsort(1, descending=True).argsort(1)
    ref = pos | (rank < (3.0 * pos.sum(1, keepdim=True)).clamp(max=P - 1))
    assert torch.equal(sel, ref)
    n_neg = (sel & ~pos).sum(1)
    want = (3 * pos.sum(1)).clamp(max=P - 1)
    assert torch.all(n_neg <= want)
    assert torch.all(n_neg[:3] == want[:3])
