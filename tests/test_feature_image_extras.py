"""D7 image-pipeline extras: Hadoop SequenceFile image sets (ImageSet.readSequenceFiles),
ImageRandomCropper, the ROI transformers and the SSD random sampler
(Zs/feature/image/{ImageSet,ImageRandomCropper,RoiTransformer,RandomSampler}.scala)."""
import numpy as np
import pytest


def test_sequence_file_roundtrip_and_read_sequence_files(tmp_path):
    from zoo.feature.image import ImageSet
    from zoo.feature.image.sequence_file import (_read_vint, _write_vint, encode_image_record,
                                                 read_sequence_file, write_sequence_file)
    for v in (0, 1, -5, 127, -112, 128, 300, -300, 70000, 2 ** 31 - 1, -2 ** 33):
        assert _read_vint(_write_vint(v), 0)[0] == v
    r = np.random.RandomState(0)
    imgs = [r.randint(0, 255, (5 + i, 7, 3)).astype(np.uint8) for i in range(6)]
    recs = [encode_image_record(i % 3 + 1 if i != 5 else 2000, "img%d.jpg" % i, im) for i, im in enumerate(imgs)]
    d = tmp_path / "seq"
    d.mkdir()
    write_sequence_file(str(d / "part-00000"), recs[:3], sync_every=64)
    write_sequence_file(str(d / "part-00001"), recs[3:], compress=True)
    assert [k for k, _ in read_sequence_file(str(d / "part-00000"))] == [k for k, _ in recs[:3]]
    s = ImageSet.read_sequence_files(str(d), class_num=1000)
    assert len(s) == 5   # label 2000 > class_num dropped
    labels = [int(f["label"][0]) for f in s.features]
    assert labels == [1, 2, 3, 1, 2]
    assert np.array_equal(s.features[4]["mat"].astype(np.uint8), imgs[4])


def _feat(h=40, w=60):
    return {"mat": np.zeros((h, w, 3), np.float32), "originalSize": (h, w, 3),
            "roi": {"classes": np.array([1, 2]), "bboxes": np.array([[6, 4, 30, 20], [40, 30, 58, 39]], np.float32)}}


def test_roi_normalize_hflip_resize_project():
    from zoo.feature.image import (ImageFixedCrop, ImageResize, ImageRoiHFlip, ImageRoiNormalize, ImageRoiProject,
                                   ImageRoiResize)
    f = ImageRoiNormalize().transform(_feat())
    assert np.allclose(f["roi"]["bboxes"][0], [0.1, 0.1, 0.5, 0.5])
    f = ImageRoiHFlip(normalized=True).transform(f)
    assert np.allclose(f["roi"]["bboxes"][0], [0.5, 0.1, 0.9, 0.5])
    g = _feat()
    g["mat"] = np.zeros((20, 120, 3), np.float32)   # resized 40x60 -> 20x120
    g = ImageRoiResize().transform(g)
    assert np.allclose(g["roi"]["bboxes"][0], [12, 2, 60, 10])
    # crop the left half: box 0 (centre inside) survives re-normalised, box 1 is dropped
    f = ImageRoiNormalize().transform(_feat())
    f = ImageFixedCrop(0.0, 0.0, 0.5, 1.0, normalized=True).transform(f)
    f = ImageRoiProject().transform(f)
    assert f["roi"]["bboxes"].shape == (1, 4) and list(f["roi"]["classes"]) == [1]
    assert np.allclose(f["roi"]["bboxes"][0], [0.2, 0.1, 1.0, 0.5])


def test_random_cropper_and_sampler():
    from zoo.feature.image import ImageRandomCropper, ImageRandomSampler, ImageRoiNormalize, ImageRoiProject
    f = {"mat": np.arange(40 * 60 * 3, dtype=np.float32).reshape(40, 60, 3), "originalSize": (40, 60, 3)}
    c = ImageRandomCropper(32, 24, mirror=True, cropper_method="center").transform(dict(f))
    assert c["mat"].shape == (24, 32, 3)
    x0 = (60 - 32) // 2
    center = f["mat"][8:32, x0:x0 + 32]
    assert np.array_equal(c["mat"], center) or np.array_equal(c["mat"], center[:, ::-1])
    for _ in range(20):
        g = ImageRandomSampler().transform(ImageRoiNormalize().transform(_feat()))
        g = ImageRoiProject().transform(g)
        h, w = g["mat"].shape[:2]
        assert 0 < h <= 40 and 0 < w <= 60
        b = g["roi"]["bboxes"]
        assert b.size == 0 or (b.min() >= 0 and b.max() <= 1)
