"""tf.data dataset graphs executed without TensorFlow (zoo.tfpark.tf_data_graph; T4,
TFDataFeatureSet.scala:31-203): slice -> map (FunctionDef) -> filter -> shuffle -> batch ->
prefetch pipelines and a TFRecord -> ParseExampleV2 pipeline, built as GraphDefs with the same
op / attr / function-library layout TensorFlow serializes (parity unpinned: no TF runtime here)."""
import numpy as np
import pytest

from zoo.util import tf as T

F32, I64, STR, BOOL = 1, 9, 7, 10


def _slice_map_graph(x, y, batch=4, shuffle=False, filter_min=None):
    # map fn: (x, y) -> (x * 2 + 1, y)
    body = [T.node_def("two", "Const", dtype=("type", F32), value=np.array(2.0, np.float32)),
            T.node_def("one", "Const", dtype=("type", F32), value=np.array(1.0, np.float32)),
            T.node_def("mul", "Mul", ["x", "two:output:0"], T=("type", F32)),
            T.node_def("add", "AddV2", ["mul:z:0", "one:output:0"], T=("type", F32))]
    fmap = T.function_def("map_fn", [("x", F32), ("y", I64)], [("x_out", F32), ("y_out", I64)], body,
                          {"x_out": "add:z:0", "y_out": "y"})
    lib = [fmap]
    nodes = [T.const_node("xs", x), T.const_node("ys", y),
             T.node_def("slice", "TensorSliceDataset", ["xs", "ys"], Toutput_types=("types", [F32, I64]),
                        output_shapes=("shapes", [list(x.shape[1:]), []])),
             T.node_def("map", "MapDataset", ["slice"], f=("func", "map_fn"), Targuments=("types", []),
                        output_types=("types", [F32, I64]))]
    last = "map"
    if filter_min is not None:
        fbody = [T.node_def("lim", "Const", dtype=("type", I64), value=np.array(filter_min, np.int64)),
                 T.node_def("ge", "GreaterEqual", ["y", "lim:output:0"], T=("type", I64))]
        lib.append(T.function_def("keep", [("x", F32), ("y", I64)], [("ok", BOOL)], fbody, {"ok": "ge:z:0"}))
        nodes.append(T.node_def("filter", "FilterDataset", [last], predicate=("func", "keep"),
                                Targuments=("types", [])))
        last = "filter"
    if shuffle:
        nodes += [T.const_node("buf", np.array(100, np.int64)), T.const_node("seed", np.array(7, np.int64)),
                  T.const_node("seed2", np.array(3, np.int64)),
                  T.node_def("shuffle", "ShuffleDataset", [last, "buf", "seed", "seed2"])]
        last = "shuffle"
    nodes += [T.const_node("bs", np.array(batch, np.int64)), T.const_node("drop", np.array(False)),
              T.node_def("batch", "BatchDatasetV2", [last, "bs", "drop"]),
              T.const_node("pf", np.array(-1, np.int64)),
              T.node_def("prefetch", "PrefetchDataset", ["batch", "pf"])]
    return T.graph_def(nodes, lib)


def test_slice_map_batch_prefetch():
    from zoo.tfpark.tf_data_graph import TFDataGraph
    x = np.arange(30, dtype=np.float32).reshape(10, 3)
    y = np.arange(10, dtype=np.int64)
    g = TFDataGraph(_slice_map_graph(x, y))
    assert g.output == "prefetch"
    batches = list(g.elements())
    assert [b[0].shape[0] for b in batches] == [4, 4, 2]
    np.testing.assert_allclose(np.concatenate([b[0] for b in batches]), x * 2 + 1)
    np.testing.assert_array_equal(np.concatenate([b[1] for b in batches]), y)
    # unbatched view: one element per row
    rows = list(g.unbatched())
    assert len(rows) == 10 and rows[3][0].shape == (3,)


def test_filter_and_shuffle():
    from zoo.tfpark.tf_data_graph import TFDataGraph
    x = np.random.rand(20, 2).astype(np.float32)
    y = np.arange(20, dtype=np.int64)
    g = TFDataGraph(_slice_map_graph(x, y, batch=5, shuffle=True, filter_min=6))
    got = np.concatenate([b[1] for b in g.elements()])
    assert sorted(got.tolist()) == list(range(6, 20))
    assert got.tolist() != list(range(6, 20))          # shuffled
    again = np.concatenate([b[1] for b in TFDataGraph(_slice_map_graph(x, y, 5, True, 6)).elements()])
    np.testing.assert_array_equal(got, again)          # seeded: reproducible


def test_tfrecord_parse_example_pipeline(tmp_path):
    from zoo.tfpark.tf_data_graph import TFDataGraph
    from zoo.tfpark.tf_dataset import TFDataset, encode_example, write_tfrecord
    recs = [encode_example({"feat": np.arange(4, dtype=np.float32) + i, "label": np.array([i % 3], np.int64)})
            for i in range(9)]
    path = str(tmp_path / "d.tfrecord")
    write_tfrecord(path, recs)
    body = [T.node_def("names", "Const", dtype=("type", STR), value=np.array([], dtype=object)),
            T.node_def("skeys", "Const", dtype=("type", STR), value=np.array([], dtype=object)),
            T.node_def("dkeys", "Const", dtype=("type", STR), value=np.array([b"feat", b"label"], dtype=object)),
            T.node_def("rkeys", "Const", dtype=("type", STR), value=np.array([], dtype=object)),
            T.node_def("d0", "Const", dtype=("type", F32), value=np.zeros(0, np.float32)),
            T.node_def("d1", "Const", dtype=("type", I64), value=np.zeros(0, np.int64)),
            T.node_def("parse", "ParseExampleV2", ["rec", "names:output:0", "skeys:output:0", "dkeys:output:0",
                                                   "rkeys:output:0", "d0:output:0", "d1:output:0"],
                       num_sparse=0, Tdense=("types", [F32, I64]), dense_shapes=("shapes", [[4], []]),
                       sparse_types=("types", []), ragged_value_types=("types", []),
                       ragged_split_types=("types", []))]
    fparse = T.function_def("parse_fn", [("rec", STR)], [("feat", F32), ("label", I64)], body,
                            {"feat": "parse:dense_values:0", "label": "parse:dense_values:1"})
    nodes = [T.const_node("files", np.array([path.encode()], dtype=object)),
             T.const_node("comp", np.array(b"", dtype=object)), T.const_node("bufsz", np.array(0, np.int64)),
             T.node_def("tfrec", "TFRecordDataset", ["files", "comp", "bufsz"]),
             T.node_def("map", "ParallelMapDatasetV2", ["tfrec", "npc"], f=("func", "parse_fn"),
                        Targuments=("types", [])),
             T.const_node("npc", np.array(-1, np.int64)),
             T.const_node("bs", np.array(4, np.int64)), T.const_node("drop", np.array(True)),
             T.node_def("batch", "BatchDatasetV2", ["map", "bs", "drop"])]
    gb = T.graph_def(nodes, [fparse])
    batches = list(TFDataGraph(gb).elements())
    assert len(batches) == 2 and batches[0][0].shape == (4, 4) and batches[0][1].shape == (4,)
    np.testing.assert_allclose(batches[1][0][0], np.arange(4) + 4)
    # the TFPark entry point takes the graph directly (trailing batch undone, FeatureSet re-batches)
    ds = TFDataset.from_tf_data_dataset(gb, batch_size=3)
    assert ds is not None


def test_unsupported_op_fails_loudly():
    from zoo.tfpark.tf_data_graph import TFDataGraph
    gb = T.graph_def([T.const_node("xs", np.zeros((2, 2), np.float32)),
                      T.node_def("fm", "FlatMapDataset", ["xs"], f=("func", "nope"))])
    with pytest.raises(NotImplementedError):
        list(TFDataGraph(gb).elements())
