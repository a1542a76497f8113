"""Image / 3D image / text pipelines and dataset loaders (ImageSetSpec,
TextSetSpec, image3d specs, test_image_set.py / test_text_set.py analogues).
Reference fixtures used read-only: pyzoo/test/zoo/resources/cat_dog (JPEGs),
zoo/src/test/resources/news20 (text folders)."""
import os

import numpy as np
import pytest
import torch

RES = "/root/reference/pyzoo/test/zoo/resources"
NEWS = "/root/reference/zoo/src/test/resources/news20"


def test_image_transforms_chain():
    from zoo.feature.common import ChainedPreprocessing
    from zoo.feature.image import (ImageCenterCrop, ImageChannelNormalize, ImageHFlip, ImageMatToTensor,
                                   ImageResize, ImageSet, ImageSetToSample, set_seed)
    set_seed(0)
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 255, (40, 50, 3)).astype(np.uint8) for _ in range(3)]
    s = ImageSet.from_arrays(imgs, labels=[1, 2, 3])
    chain = ChainedPreprocessing([ImageResize(32, 32), ImageCenterCrop(24, 24), ImageHFlip(),
                                  ImageChannelNormalize(100.0, 110.0, 120.0, 2.0, 2.0, 2.0),
                                  ImageMatToTensor(), ImageSetToSample()])
    out = s.transform(chain)
    t = out.features[0]["imageTensor"]
    assert t.shape == (3, 24, 24)
    # independent check of the same pipeline on image 0
    from zoo.feature.image.transforms import resize_bilinear
    m = resize_bilinear(imgs[0].astype(np.float32), 32, 32)[4:28, 4:28][:, ::-1]
    m = (m - np.array([120.0, 110.0, 100.0])) / 2.0
    assert np.allclose(t, m.transpose(2, 0, 1), atol=1e-4)
    fs = out.to_featureset(batch_size=2, shuffle=False)
    xb, yb = next(iter(fs.data(train=False)))
    assert tuple(xb.shape) == (2, 3, 24, 24) and yb.tolist() == [1.0, 2.0]


def test_resize_matches_pil_bilinear_shape_and_identity():
    from zoo.feature.image.transforms import resize_bilinear
    a = np.arange(2 * 3 * 1, dtype=np.float32).reshape(2, 3, 1)
    assert np.allclose(resize_bilinear(a, 2, 3), a)
    up = resize_bilinear(a, 4, 6)
    assert up.shape == (4, 6, 1) and up.min() >= a.min() and up.max() <= a.max()


@pytest.mark.skipif(not os.path.isdir(os.path.join(RES, "cat_dog")), reason="fixture missing")
def test_imageset_read_with_labels():
    from zoo.feature.image import ImageAspectScale, ImageSet
    s = ImageSet.read(os.path.join(RES, "cat_dog"), with_label=True, one_based_label=True)
    assert len(s) >= 2 and s.label_map == {"cats": 1, "dogs": 2}
    labels = sorted({float(l[0]) for l in s.get_label()})
    assert labels == [1.0, 2.0]
    s2 = s.transform(ImageAspectScale(64, max_size=200))
    assert min(s2.features[0]["mat"].shape[:2]) == 64 or max(s2.features[0]["mat"].shape[:2]) == 200


def test_color_ops_keep_shape_and_range():
    from zoo.feature.image import ImageColorJitter, ImageExpand, ImageSet, set_seed
    set_seed(3)
    rng = np.random.default_rng(1)
    s = ImageSet.from_arrays([rng.integers(0, 255, (16, 16, 3)).astype(np.uint8)])
    j = s.transform(ImageColorJitter(1.0, 16, 1.0, 0.8, 1.2, 1.0, 10, 1.0, 0.8, 1.2))
    assert j.features[0]["mat"].shape == (16, 16, 3)
    e = s.transform(ImageExpand(min_expand_ratio=2.0, max_expand_ratio=2.0))
    assert e.features[0]["mat"].shape == (32, 32, 3)


def test_image3d_affine_and_crop():
    from zoo.feature.image3d import AffineTransform3D, Crop3D, ImageFeature3D, Rotate3D
    vol = np.random.default_rng(0).random((6, 7, 8)).astype(np.float32)
    f = AffineTransform3D(np.eye(3)).transform(ImageFeature3D(vol.copy()))
    assert np.allclose(f["image"], vol, atol=1e-5)
    c = Crop3D([1, 2, 3], [2, 3, 4]).transform(ImageFeature3D(vol.copy()))
    assert np.array_equal(c["image"], vol[1:3, 2:5, 3:7])
    # rotating by pi about the depth axis twice restores the volume
    r = Rotate3D([np.pi, 0, 0]).transform(Rotate3D([np.pi, 0, 0]).transform(ImageFeature3D(vol.copy())))
    assert np.allclose(r["image"][1:-1, 1:-1, 1:-1], vol[1:-1, 1:-1, 1:-1], atol=1e-4)


def test_textset_pipeline_and_word_index(tmp_path):
    from zoo.feature.text import TextSet
    ts = TextSet.from_texts(["Hello World hello", "world of zoo!", "zoo zoo zoo"], labels=[0, 1, 1])
    ts = ts.tokenize().normalize()
    assert ts.features[1]["tokens"] == ["world", "of", "zoo"]
    ts = ts.word2idx(remove_topN=1)  # drop "zoo" (most frequent)
    wi = ts.get_word_index()
    assert "zoo" not in wi and wi["hello"] == 1 and wi["world"] == 2
    ts = ts.shape_sequence(4, trunc_mode="post").generate_sample()
    assert ts.features[0]["indices"].tolist() == [1.0, 2.0, 1.0, 0.0]
    assert ts.features[2]["indices"].tolist() == [0.0, 0.0, 0.0, 0.0]
    p = str(tmp_path / "wi.txt")
    ts.save_word_index(p)
    assert TextSet.from_texts(["x"]).load_word_index(p).get_word_index() == wi
    fs = ts.to_featureset(batch_size=3, shuffle=False)
    xb, yb = next(iter(fs.data(train=False)))
    assert tuple(xb.shape) == (3, 4) and yb.tolist() == [0.0, 1.0, 1.0]
    a, b = ts.random_split([0.5, 0.5], seed=1)
    assert len(a) + len(b) == 3


def test_relation_pairs_and_lists():
    from zoo.feature.text import Relation, TextSet
    q = TextSet.from_texts(["a b", "c d"]).tokenize().word2idx()
    q.features[0]["uri"], q.features[1]["uri"] = "q1", "q2"
    q = q.shape_sequence(2)
    a = TextSet.from_texts(["x", "y", "z"]).tokenize().word2idx().shape_sequence(3)
    for i, u in enumerate(["a1", "a2", "a3"]):
        a.features[i]["uri"] = u
    rel = [Relation("q1", "a1", 1), Relation("q1", "a2", 0), Relation("q1", "a3", 0), Relation("q2", "a3", 1)]
    pairs = TextSet.from_relation_pairs(rel, q, a)
    assert len(pairs) == 2
    feat, lab = pairs.features[0]["sample"]
    assert feat.shape == (2, 5) and lab.tolist() == [[1.0], [0.0]]
    lists = TextSet.from_relation_lists(rel, q, a)
    assert lists.features[0]["sample"][0].shape == (3, 5)


@pytest.mark.skipif(not os.path.isdir(NEWS), reason="fixture missing")
def test_textset_read_folders():
    from zoo.feature.text import TextSet
    ts = TextSet.read(NEWS)
    assert len(ts) == 5 and sorted(set(ts.get_labels())) == [0, 1, 2]  # alt.atheism, rec.autos, sci.space


def test_mnist_idx_roundtrip(tmp_path):
    from zoo.pipeline.api.keras.datasets import mnist
    x = np.random.default_rng(0).integers(0, 255, (5, 28, 28)).astype(np.uint8)
    y = np.arange(5, dtype=np.uint8)
    for name, arr in (("train-images-idx3-ubyte.gz", x), ("train-labels-idx1-ubyte.gz", y),
                      ("t10k-images-idx3-ubyte", x[:2]), ("t10k-labels-idx1-ubyte", y[:2])):
        mnist.write_idx(str(tmp_path / name), arr)
    (xt, yt), (xe, ye) = mnist.load_data(str(tmp_path))
    assert np.array_equal(xt, x) and np.array_equal(yt, y) and xe.shape == (2, 28, 28)


def test_imdb_npz_and_boston(tmp_path):
    from zoo.pipeline.api.keras.datasets import boston_housing, imdb
    np.savez(tmp_path / "imdb.npz", x_train=np.array([[5, 6, 0], [7, 0, 0]]), y_train=np.array([1, 0]),
             x_test=np.array([[8, 9, 10]]), y_test=np.array([1]))
    (xtr, ytr), (xte, yte) = imdb.load_data(str(tmp_path), nb_words=11)
    assert xtr[0].tolist() == [1, 8, 9] and xtr[1].tolist() == [1, 10] and xte[0].tolist() == [1, 2, 2, 2]
    np.savez(tmp_path / "boston_housing.npz", x=np.random.rand(10, 13), y=np.random.rand(10))
    (a, b), (c, d) = boston_housing.load_data(str(tmp_path))
    assert a.shape == (8, 13) and c.shape == (2, 13)


@pytest.mark.gpu
def test_gpu_resize_normalize_kernel(gpu):
    from zoo.feature.image.transforms import gpu_resize_normalize, resize_bilinear
    rng = np.random.default_rng(0)
    batch = rng.integers(0, 255, (3, 37, 53, 3)).astype(np.uint8)
    out = gpu_resize_normalize(batch, 24, 32, mean=(10.0, 20.0, 30.0), std=(2.0, 3.0, 4.0), swap_rb=True,
                               layout="NCHW", device=gpu)
    ref = np.stack([resize_bilinear(b.astype(np.float32), 24, 32)[..., ::-1] for b in batch])
    ref = (ref - np.array([10.0, 20.0, 30.0])) / np.array([2.0, 3.0, 4.0])
    assert np.allclose(out.cpu().numpy(), ref.transpose(0, 3, 1, 2), atol=1e-3)
    nhwc = gpu_resize_normalize(batch, 24, 32, layout="NHWC4", device=gpu)
    assert tuple(nhwc.shape) == (3, 24, 32, 4) and nhwc.dtype == torch.bfloat16
    assert float(nhwc[..., 3].abs().max()) == 0.0
    ref2 = np.stack([resize_bilinear(b.astype(np.float32), 24, 32) for b in batch])
    assert np.allclose(nhwc[..., :3].float().cpu().numpy(), ref2, rtol=1e-2, atol=1.0)
