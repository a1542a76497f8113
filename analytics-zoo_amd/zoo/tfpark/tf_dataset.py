"""TFDataset (Py/tfpark/tf_dataset.py:TFDataset.from_*) -> FeatureSet."""
import numpy as np

from zoo.feature.common import FeatureSet


class TFDataset:
    def __init__(self, train, val=None, batch_size=32, batch_per_thread=-1, hard_code_batch_size=False):
        self.train, self.val = train, val
        self.batch_size, self.batch_per_thread = batch_size, batch_per_thread

    def get_training_data(self):
        return self.train

    def get_validation_data(self):
        return self.val

    def get_prediction_data(self):
        return self.train

    def get_evaluation_data(self):
        return self.val or self.train

    def get_num_partitions(self):
        from zoo.common.nncontext import get_nncontext
        return get_nncontext().world_size

    @staticmethod
    def _bs(batch_size, batch_per_thread):
        return batch_size if batch_size and batch_size > 0 else (batch_per_thread if batch_per_thread > 0 else 32)

    @staticmethod
    def from_ndarrays(tensors, batch_size=-1, batch_per_thread=-1, hard_code_batch_size=False, val_tensors=None,
                      memory_type="DRAM"):
        bs = TFDataset._bs(batch_size, batch_per_thread)
        x, y = (tensors[0], tensors[1]) if isinstance(tensors, tuple) and len(tensors) == 2 else (tensors, None)
        train = FeatureSet.from_ndarrays(x, y, bs, shuffle=batch_size > 0)
        val = None
        if val_tensors is not None:
            vx, vy = val_tensors if isinstance(val_tensors, tuple) else (val_tensors, None)
            val = FeatureSet.from_ndarrays(vx, vy, bs, shuffle=False)
        return TFDataset(train, val, batch_size, batch_per_thread)

    @staticmethod
    def from_feature_set(dataset, features=None, labels=None, batch_size=-1, batch_per_thread=-1,
                         hard_code_batch_size=False, validation_dataset=None):
        return TFDataset(dataset, validation_dataset, batch_size, batch_per_thread)

    @staticmethod
    def from_image_set(image_set, image=None, label=None, batch_size=-1, batch_per_thread=-1,
                       hard_code_batch_size=False, validation_image_set=None):
        bs = TFDataset._bs(batch_size, batch_per_thread)
        val = validation_image_set.to_featureset(bs, shuffle=False) if validation_image_set is not None else None
        return TFDataset(image_set.to_featureset(bs, shuffle=batch_size > 0), val, batch_size, batch_per_thread)

    @staticmethod
    def from_text_set(text_set, text=None, label=None, batch_size=-1, batch_per_thread=-1,
                      hard_code_batch_size=False, validation_text_set=None):
        bs = TFDataset._bs(batch_size, batch_per_thread)
        val = validation_text_set.to_featureset(bs, shuffle=False) if validation_text_set is not None else None
        return TFDataset(text_set.to_featureset(bs, shuffle=batch_size > 0), val, batch_size, batch_per_thread)

    @staticmethod
    def from_dataframe(df, feature_cols, labels_cols=None, batch_size=-1, batch_per_thread=-1,
                       hard_code_batch_size=False, validation_df=None):
        bs = TFDataset._bs(batch_size, batch_per_thread)

        def arrays(d):
            x = np.stack([np.concatenate([np.asarray(r[c], np.float32).reshape(-1) for c in feature_cols])
                          for _, r in d.iterrows()])
            y = None
            if labels_cols:
                y = np.stack([np.concatenate([np.asarray(r[c], np.float32).reshape(-1) for c in labels_cols])
                              for _, r in d.iterrows()])
                y = y[:, 0] if y.shape[1] == 1 else y
            return x, y
        x, y = arrays(df)
        val = FeatureSet.from_ndarrays(*arrays(validation_df), bs, shuffle=False) if validation_df is not None \
            else None
        return TFDataset(FeatureSet.from_ndarrays(x, y, bs, shuffle=batch_size > 0), val, batch_size,
                         batch_per_thread)

    @staticmethod
    def from_tf_data_dataset(dataset, batch_size=-1, batch_per_thread=-1, hard_code_batch_size=False,
                             validation_dataset=None, sequential_order=False, shuffle=True):
        """Py/tfpark/tf_dataset.py:TFDataDataset (T4 TFDataFeatureSet). ``dataset`` is a tf.data
        pipeline as its serialized dataset graph -- GraphDef bytes, a path to one, or a
        ``tf.data.Dataset`` (``_as_serialized_graph``) -- executed by zoo.tfpark.tf_data_graph
        (a trailing batch is undone: the FeatureSet batches), or any iterable of UNBATCHED
        elements ``x`` / ``(x, y)``. Elements are materialised once into host arrays and served
        by the native FeatureSet gather."""
        from zoo.tfpark.tf_data_graph import TFDataGraph, serialized_graph
        bs = TFDataset._bs(batch_size, batch_per_thread)

        def from_graph(d):
            gb = serialized_graph(d) if d is not None and not isinstance(d, (list, tuple)) else None
            if gb is None:
                return d
            return [e[0] if len(e) == 1 else tuple(e) for e in TFDataGraph(gb).unbatched()]
        dataset, validation_dataset = from_graph(dataset), from_graph(validation_dataset)
        train = _iterable_featureset(dataset, bs, shuffle and not sequential_order and batch_size > 0)
        val = _iterable_featureset(validation_dataset, bs, False) if validation_dataset is not None else None
        return TFDataset(train, val, batch_size, batch_per_thread)

    @staticmethod
    def from_tfrecord_file(file_path, batch_size=-1, batch_per_thread=-1, hard_code_batch_size=False,
                           validation_file_path=None, parse_fn=None, feature_keys=None, label_key=None):
        """Py/tfpark/tf_dataset.py:TFRecordDataset. Records are read with the native TFRecord
        framing and decoded as ``tf.train.Example`` protos (:func:`parse_example`). ``parse_fn``
        maps the decoded ``{name: ndarray}`` dict to ``x`` or ``(x, y)`` (the reference maps
        the serialized string with TF ops instead); by default the ``feature_keys`` features
        are concatenated into x and ``label_key`` is y."""
        bs = TFDataset._bs(batch_size, batch_per_thread)

        def elements(path):
            paths = path if isinstance(path, (list, tuple)) else [path]
            for pth in paths:
                for rec in read_tfrecord(pth):
                    ex = parse_example(rec)
                    if parse_fn is not None:
                        yield parse_fn(ex)
                        continue
                    keys = feature_keys or sorted(k for k in ex if k != label_key)
                    x = np.concatenate([np.asarray(ex[k], np.float32).reshape(-1) for k in keys])
                    yield (x, ex[label_key]) if label_key is not None else x
        train = _iterable_featureset(elements(file_path), bs, batch_size > 0)
        val = _iterable_featureset(elements(validation_file_path), bs, False) \
            if validation_file_path is not None else None
        return TFDataset(train, val, batch_size, batch_per_thread)

    @staticmethod
    def from_rdd(rdd, names=None, shapes=None, types=None, batch_size=-1, batch_per_thread=-1,
                 hard_code_batch_size=False, val_rdd=None, memory_type="DRAM", sequential_order=False,
                 shuffle=True):
        """Py/tfpark/tf_dataset.py:1016 (TFNdarrayDataset over an RDD of samples): ``rdd`` is any
        collection of ``x`` or ``(x, y)`` samples -- a list / iterable, an XShards/``RayRDD``-like
        object with ``collect()``, or a FeatureSet (then used as is)."""
        if isinstance(rdd, FeatureSet):
            return TFDataset.from_feature_set(rdd, batch_size=batch_size, batch_per_thread=batch_per_thread,
                                              validation_dataset=val_rdd)
        bs = TFDataset._bs(batch_size, batch_per_thread)
        train = _iterable_featureset(_collect(rdd), bs, shuffle and not sequential_order and batch_size > 0)
        val = _iterable_featureset(_collect(val_rdd), bs, False) if val_rdd is not None else None
        return TFDataset(train, val, batch_size, batch_per_thread)

    @staticmethod
    def from_string_rdd(string_rdd, batch_size=-1, batch_per_thread=-1, hard_code_batch_size=False,
                        validation_string_rdd=None):
        """Py/tfpark/tf_dataset.py:528: a dataset of single strings (utf-8 encoded to bytes);
        batches are ``(list_of_bytes,)`` -- the reference's one tf.string feature tensor of
        shape (None,). Labels, if any, live inside the strings."""
        enc = (lambda v: v.encode("utf-8") if isinstance(v, str) else bytes(v))
        val = None if validation_string_rdd is None else [enc(v) for v in _collect(validation_string_rdd)]
        return TFDataset.from_bytes_rdd([enc(v) for v in _collect(string_rdd)], batch_size, batch_per_thread,
                                        hard_code_batch_size, val)

    @staticmethod
    def from_bytes_rdd(bytes_rdd, batch_size=-1, batch_per_thread=-1, hard_code_batch_size=False,
                       validation_bytes_rdd=None):
        """Py/tfpark/tf_dataset.py:553 (TFBytesDataset): a dataset of byte strings served in
        batches of ``(list_of_bytes,)`` (shuffled per epoch for training)."""
        bs = TFDataset._bs(batch_size, batch_per_thread)
        train = BytesFeatureSet(list(_collect(bytes_rdd)), bs, shuffle=batch_size > 0,
                                drop_last=hard_code_batch_size)
        val = BytesFeatureSet(list(_collect(validation_bytes_rdd)), bs, shuffle=False) \
            if validation_bytes_rdd is not None else None
        return TFDataset(train, val, batch_size, batch_per_thread)


def _collect(rdd):
    """An 'RDD' here: a list/iterable, or anything with collect() (XShards, RayRDD)."""
    if hasattr(rdd, "collect"):
        rdd = rdd.collect()
    return list(rdd)


class BytesFeatureSet(FeatureSet):
    """Variable-length byte records (TFBytesDataset): batches are ``(list_of_bytes,)``."""

    def __init__(self, records, batch_size=32, shuffle=True, drop_last=False, seed=0):
        self.records = [bytes(r) for r in records]
        self.batch_size, self.shuffle, self.drop_last, self.seed = int(batch_size), shuffle, drop_last, seed

    def size(self):
        return len(self.records)

    def data(self, train=True, epoch=None):
        idx = np.arange(len(self.records))
        if train and self.shuffle:
            np.random.default_rng(self.seed + (epoch or 0)).shuffle(idx)
        n = len(idx)
        stop = n - n % self.batch_size if (self.drop_last and train) else n
        for s in range(0, stop, self.batch_size):
            yield ([self.records[i] for i in idx[s:s + self.batch_size]],)


def _iterable_featureset(dataset, batch_size, shuffle):
    it = dataset.as_numpy_iterator() if hasattr(dataset, "as_numpy_iterator") else iter(dataset)
    xs, ys = [], []
    for el in it:
        if isinstance(el, dict):
            raise TypeError("dict elements: map them to x or (x, y) first")
        if isinstance(el, (tuple, list)) and len(el) == 2:
            xs.append(np.asarray(el[0]))
            ys.append(np.asarray(el[1]))
        else:
            xs.append(np.asarray(el))
    if not xs:
        raise ValueError("the dataset is empty")
    x = np.stack(xs)
    y = None
    if ys:
        y = np.stack(ys)
        if y.ndim == 2 and y.shape[1] == 1:
            y = y[:, 0]
    return FeatureSet.from_ndarrays(x, y, batch_size, shuffle=shuffle)


# ---- tf.train.Example (example.proto / feature.proto) codec, no TensorFlow needed ----
def _packed(v, wt, kind):
    if wt != 2:  # unpacked scalar element
        if kind == "f":
            return [np.frombuffer(int(v).to_bytes(4, "little"), np.float32)[0]]
        return [v - (1 << 64) if v >= 1 << 63 else v]
    if kind == "f":
        return list(np.frombuffer(v, np.float32))
    from zoo.utils.protobuf import _varint
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x - (1 << 64) if x >= 1 << 63 else x)
    return out


def parse_example(record):
    """Serialized ``tf.train.Example`` -> {name: ndarray} (bytes_list -> object array of
    bytes, float_list -> float32, int64_list -> int64)."""
    from zoo.utils.protobuf import fields
    out = {}
    for f, _, feats in fields(record):
        if f != 1:
            continue
        for ff, _, entry in fields(feats):
            if ff != 1:
                continue
            key, feat = "", b""
            for ef, _, ev in fields(entry):
                if ef == 1:
                    key = ev.decode("utf-8")
                elif ef == 2:
                    feat = ev
            arr = np.zeros((0,), np.float32)
            for kind, _, lst in fields(feat):
                vals = [(wt, v) for vf, wt, v in fields(lst) if vf == 1]
                if kind == 1:
                    arr = np.array([v for _, v in vals], dtype=object)
                elif kind == 2:
                    arr = np.array([x for wt, v in vals for x in _packed(v, wt, "f")], np.float32)
                elif kind == 3:
                    arr = np.array([x for wt, v in vals for x in _packed(v, wt, "i")], np.int64)
            out[key] = arr
    return out


def encode_example(features):
    """{name: bytes | str | float/int array} -> serialized ``tf.train.Example``."""
    from zoo.tensorboard import _field, _varint
    entries = b""
    for key in sorted(features):
        v = features[key]
        if isinstance(v, (bytes, str)) or (isinstance(v, (list, tuple)) and v and isinstance(v[0], (bytes, str))):
            items = [v] if isinstance(v, (bytes, str)) else list(v)
            lst = b"".join(_field(1, 2, x.encode() if isinstance(x, str) else x) for x in items)
            feat = _field(1, 2, lst)
        else:
            a = np.asarray(v).reshape(-1)
            if np.issubdtype(a.dtype, np.floating):
                feat = _field(2, 2, _field(1, 2, a.astype("<f4").tobytes()))
            else:
                packed = b"".join(_varint(int(x) & ((1 << 64) - 1)) for x in a)
                feat = _field(3, 2, _field(1, 2, packed))
        entries += _field(1, 2, _field(1, 2, key.encode()) + _field(2, 2, feat))
    return _field(1, 2, entries)


def read_tfrecord(path):
    from zoo.tensorboard import read_records
    return read_records(path)


def write_tfrecord(path, records):
    from zoo.tensorboard import _frame
    with open(path, "wb") as f:
        for r in records:
            f.write(_frame(r))
