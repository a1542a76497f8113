"""Utility surfaces of the reference: Py/util/nest.py, Py/common/utils.py
(paths, remote files, JTensor, Sample), Zs/utils/File.scala (FS helpers)."""
import collections
import os

import numpy as np
import pytest

from zoo.util import nest
from zoo.utils import file as zfile
from zoo.common import utils as cu


def test_nest_flatten_and_pack_roundtrip():
    Pt = collections.namedtuple("Pt", "x y")
    s = {"b": [1, (2, 3)], "a": Pt(4, {"z": 5, "y": 6})}
    flat = nest.flatten(s)
    assert flat == [4, 6, 5, 1, 2, 3]   # dicts flatten in sorted-key order
    back = nest.pack_sequence_as(s, [v * 10 for v in flat])
    assert back == {"b": [10, (20, 30)], "a": Pt(40, {"z": 50, "y": 60})}
    assert nest.flatten(7) == [7] and nest.pack_sequence_as(0, [9]) == 9
    with pytest.raises(ValueError):
        nest.pack_sequence_as([1, 2], [1])


def test_file_helpers_local_and_file_uri(tmp_path):
    p = str(tmp_path / "d" / "x.bin")
    zfile.save_bytes(b"abc", p)
    assert zfile.exists(p) and zfile.read_bytes("file://" + p) == b"abc"
    with pytest.raises(FileExistsError):
        zfile.save_bytes(b"zz", p)
    zfile.save_bytes(b"zz", "file://" + p, overwrite=True)
    assert zfile.read_bytes(p) == b"zz"
    assert zfile.list_files(str(tmp_path / "d")) == [p]
    q = str(tmp_path / "copy.bin")
    zfile.get_remote_file_to_local("file://" + p, q)
    assert open(q, "rb").read() == b"zz"
    zfile.delete(str(tmp_path / "d"))
    assert not os.path.exists(p)
    assert zfile.is_local_path("/a/b") and zfile.is_local_path("file:///a") and not zfile.is_local_path("hdfs://n/a")


def test_remote_scheme_without_client_is_explicit(monkeypatch):
    monkeypatch.setenv("PATH", "")
    with pytest.raises(NotImplementedError):
        zfile.exists("hdfs://namenode:9000/x")
    monkeypatch.delenv("AWS_ACCESS_KEY_ID", raising=False)
    monkeypatch.delenv("ZOO_S3_ENDPOINT", raising=False)
    monkeypatch.delenv("AWS_ENDPOINT_URL", raising=False)
    from zoo.utils import s3
    s3.reset_client()
    with pytest.raises(s3.S3ConfigError, match="AWS_ACCESS_KEY_ID"):   # s3 needs credentials, fails fast
        zfile.exists("s3://bucket/x")
    s3.reset_client()
    with pytest.raises(NotImplementedError):
        zfile.exists("gs://bucket/x")


def test_common_utils_save_load_and_carriers(tmp_path):
    p = str(tmp_path / "m.npy")
    cu.save_file(lambda f: np.save(f, np.arange(3)), p)
    assert cu.load_from_file(np.load, p).tolist() == [0, 1, 2]
    assert cu.append_suffix("abc", "hdfs://x/y/model.npy") == "abc.npy"
    assert [a.tolist() for a in cu.to_list_of_numpy([1, np.ones(2)])] == [1, [1.0, 1.0]]
    with pytest.raises(ValueError):
        cu.to_list_of_numpy({"a": 1})
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    assert np.array_equal(cu.JTensor.from_ndarray(a).to_ndarray(), a)
    sp = cu.JTensor.sparse(np.array([1.0, 2.0]), np.array([0, 1, 2, 0]), (2, 3))
    assert sp.to_ndarray().tolist() == [[0, 0, 1.0], [2.0, 0, 0]]
    s = cu.Sample.from_ndarray(a, np.array(1))
    assert s.feature.shape == (2, 3) and int(s.label) == 1
    with pytest.raises(NotImplementedError):
        cu.callZooFunc("float", "anything")


def test_checkpoint_file_uri(tmp_path):
    from zoo.utils.checkpoint import load_object, save_object
    import torch
    uri = "file://" + str(tmp_path / "ck" / "model.1")
    save_object({"w": torch.ones(2)}, uri)
    assert load_object(uri)["w"].tolist() == [1.0, 1.0]


REFERENCE_IMPORT_PATHS = [
    "zoo.automl.model.Seq2Seq", "zoo.automl.model.VanillaLSTM", "zoo.feature.image.imagePreprocessing",
    "zoo.feature.text.text_feature", "zoo.feature.text.transformer", "zoo.models.image.common.image_config",
    "zoo.models.image.common.image_model", "zoo.models.image.imageclassification.image_classification",
    "zoo.models.image.objectdetection.object_detector", "zoo.pipeline.api.keras.layers.convolutional_recurrent",
    "zoo.pipeline.api.keras.layers.local", "zoo.pipeline.api.keras.layers.noise",
    "zoo.pipeline.api.keras.layers.torch", "zoo.pipeline.api.keras2.layers.convolutional",
    "zoo.pipeline.api.keras2.layers.core", "zoo.pipeline.api.keras2.layers.merge",
    "zoo.pipeline.api.keras2.layers.pooling", "zoo.pipeline.api.net.net_load", "zoo.pipeline.api.net.torch_criterion",
    "zoo.pipeline.nnframes.nn_image_schema", "zoo.ray.mxnet.mxnet_trainer", "zoo.tfpark.estimator",
    "zoo.tfpark.zoo_optimizer", "zoo.tfpark.text.estimator", "zoo.tfpark.text.keras", "zoo.util.nest",
    "zoo.common.utils", "zoo.automl.search.abstract",
]


@pytest.mark.parametrize("mod", REFERENCE_IMPORT_PATHS)
def test_reference_import_paths(mod):
    """A user of the reference can keep its import paths (Py/<path>.py)."""
    import importlib
    m = importlib.import_module(mod)
    assert [n for n in dir(m) if not n.startswith("_")]


def test_layers_star_import_does_not_shadow_torch():
    import torch
    import zoo.pipeline.api.keras.layers.torch  # noqa: F401  (reference-named submodule)
    ns = {}
    exec("from zoo.pipeline.api.keras.layers import *", ns)
    assert "torch" not in ns and "Dense" in ns
    assert torch.zeros(1).numel() == 1


def test_xshard_reference_import_paths(tmp_path):
    import pandas as pd
    import zoo.xshard.pandas
    from zoo.xshard.shard import RayDataShards, RayPartition
    from zoo.xshard.pandas.preprocessing import RayPandasShard, read_file_ray
    from zoo.xshard.utils import chunk, flatten
    for i in range(3):
        pd.DataFrame({"a": [i, i + 1], "b": [1.0, 2.0]}).to_csv(tmp_path / ("p%d.csv" % i), index=False)
    sh = zoo.xshard.pandas.read_csv(str(tmp_path), None)
    assert isinstance(sh, RayDataShards) and len(sh.collect()) == 3
    out = sh.apply(lambda df, k: df.assign(c=df.a * k), 2).collect()
    assert list(out[2].c) == [4, 6]
    assert len(read_file_ray(None, str(tmp_path), "csv").collect()) == 3
    s = RayPandasShard()
    s.read_file_partitions([str(tmp_path / "p0.csv")], "csv")
    s.apply(lambda df: df[df.a > 0])
    assert len(s.get_data()) == 1
    assert RayPartition([s]).get_data()[0] is s.get_data()
    assert chunk(list(range(7)), 3) == [[0, 1, 2], [3, 4], [5, 6]] and flatten([[1], [2, 3]]) == [1, 2, 3]
