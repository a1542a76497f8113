"""FeatureSet and the Preprocessing algebra (data layer).

FeatureSet (Zs/feature/FeatureSet.scala:53-709, Py/feature/common.py:92-379):
``data(train=True)`` yields shuffled minibatches forever-per-epoch in training
and one ordered pass in evaluation. Memory tiers, MI355X-first:

  * ``DEVICE`` — the whole dataset lives in HBM (288 GB per GPU); batches are
    gathered on the GPU by index (no host traffic at all). New tier.
  * ``DRAM`` — host arrays; the native C++ Gatherer (zoo._runtime) assembles
    the next batches into pinned buffers on worker threads while the GPU runs
    the current one, then a non-blocking DMA moves them to HBM.
  * ``DIRECT`` / ``PMEM`` — same as DRAM but the arrays are copied into pinned
    (page-locked) memory once (the reference's off-heap DIRECT/PMEM tiers,
    Zs/feature/pmem/*).
  * ``DISK_AND_DRAM(n)`` — arrays memory-mapped from disk; each "slice epoch"
    stages 1/n of the shuffled data into DRAM (DiskFeatureSet, FeatureSet.scala:564-641).

Distributed sharding: every rank draws the same per-epoch permutation (seeded
by the epoch) and takes an equal-sized disjoint shard, so all ranks run the
same number of iterations (required for the synchronous collectives). The
``batch_size`` is global (as in the reference); each rank gets batch/world.
"""
import math
import os
import threading

import numpy as np
import torch


class MemoryType:
    DRAM = "DRAM"
    DEVICE = "DEVICE"
    DIRECT = "DIRECT"
    PMEM = "PMEM"

    @staticmethod
    def DISK_AND_DRAM(num_slice):  # noqa: N802 - reference name
        return "DISK_AND_DRAM_%d" % int(num_slice)


class DataStrategy:
    PARTITIONED = "PARTITIONED"
    REPLICATED = "REPLICATED"
    # the arrays ARE this rank's partition (a Spark DataFrame partition living on its executor):
    # no further sharding; every rank must hold the same number of samples (checked)
    LOCAL = "LOCAL"


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def _device():
    try:
        from zoo.common.nncontext import get_nncontext
        return get_nncontext().device
    except Exception:  # noqa: BLE001
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")


_GATHERER = None
_GLOCK = threading.Lock()


def _gatherer():
    global _GATHERER
    with _GLOCK:
        if _GATHERER is None:
            try:
                import zoo._runtime as R
                _GATHERER = R.Gatherer(int(os.environ.get("ZOO_LOADER_THREADS", "4")))
            except ImportError:
                _GATHERER = False
    return _GATHERER or None


class FeatureSet:
    """Base: subclasses implement ``data(train, epoch)`` and ``size()``."""

    def data(self, train=True, epoch=None):
        raise NotImplementedError

    def size(self):
        raise NotImplementedError

    def num_of_slice(self):
        return 1

    def transform(self, preprocessing):
        return TransformedFeatureSet(self, preprocessing)

    def __iter__(self):
        return self.data(train=False)

    def to_dataset(self):
        return self

    # ---------------------------------------------------------------- factories
    @staticmethod
    def from_ndarrays(x, y=None, batch_size=32, shuffle=True, memory_type=MemoryType.DRAM,
                      data_strategy=DataStrategy.PARTITIONED, drop_last=True):
        return ArrayFeatureSet(x, y, batch_size, shuffle, memory_type, data_strategy, drop_last)

    @staticmethod
    def ndarrays(x, y=None, batch_size=32, **kw):
        return FeatureSet.from_ndarrays(x, y, batch_size, **kw)

    @staticmethod
    def from_dataloader(loader):
        return DataLoaderFeatureSet(loader)

    @staticmethod
    def pytorch_dataloader(dataloader, features="_data[0]", labels="_data[1]"):
        """PythonLoaderFeatureSet (FeatureSet.scala:332-554): a torch DataLoader as a FeatureSet."""
        return DataLoaderFeatureSet(dataloader)

    @staticmethod
    def from_generator(fn, size=None):
        return GeneratorFeatureSet(fn, size)

    @staticmethod
    def rdd(data, memory_type=MemoryType.DRAM, data_strategy=DataStrategy.PARTITIONED, batch_size=32):
        """Reference entry point taking an RDD; here any iterable of (x, y) samples."""
        samples = list(data)
        xs = np.stack([np.asarray(s[0]) for s in samples])
        ys = np.stack([np.asarray(s[1]) for s in samples]) if len(samples[0]) > 1 else None
        return ArrayFeatureSet(xs, ys, batch_size, True, memory_type, data_strategy, True)


def _as_list(a):
    return list(a) if isinstance(a, (list, tuple)) else [a]


class ArrayFeatureSet(FeatureSet):
    def __init__(self, x, y=None, batch_size=32, shuffle=True, memory_type=MemoryType.DRAM,
                 data_strategy=DataStrategy.PARTITIONED, drop_last=True):
        self.multi_x = isinstance(x, (list, tuple))
        self.xs = [self._to_np(a) for a in _as_list(x)]
        self.ys = None if y is None else [self._to_np(a) for a in _as_list(y)]
        self.multi_y = isinstance(y, (list, tuple))
        self.n = self.xs[0].shape[0]
        for a in self.xs + (self.ys or []):
            if a.shape[0] != self.n:
                raise ValueError("all arrays must have the same number of samples")
        self.batch_size = int(batch_size)
        self.shuffle_ = shuffle
        self.memory_type = memory_type
        self.strategy = data_strategy
        self.drop_last = drop_last
        self.world, self.rank = _world()
        if self.strategy == DataStrategy.REPLICATED:
            self.world, self.rank = 1, 0
        self.local_bs = max(1, self.batch_size // self.world)
        self.presharded = self.strategy == DataStrategy.LOCAL
        if self.presharded and self.world > 1:
            self._check_equal_partitions()
        self._slices = 1
        self._dev_arrays = None
        self._pinned = None
        if memory_type.startswith("DISK_AND_DRAM"):
            self._slices = int(memory_type.rsplit("_", 1)[1])
        if memory_type == MemoryType.DEVICE:
            dev = _device()
            self._dev_arrays = [torch.from_numpy(a).to(dev) for a in self.xs + (self.ys or [])]
        elif memory_type in (MemoryType.DIRECT, MemoryType.PMEM) and torch.cuda.is_available():
            self._pinned = [torch.from_numpy(a).pin_memory() for a in self.xs + (self.ys or [])]

    @staticmethod
    def _to_np(a):
        if isinstance(a, torch.Tensor):
            a = a.detach().cpu().numpy()
        a = np.asarray(a)
        if a.dtype == np.float64:
            a = a.astype(np.float32)
        return np.ascontiguousarray(a)

    def _check_equal_partitions(self):
        """The synchronous collectives need every rank to run the same number of iterations."""
        import torch.distributed as dist
        dev = _device() if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([self.n, -self.n], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        hi, lo = int(t[0]), -int(t[1])
        if hi != lo:
            raise ValueError("DataStrategy.LOCAL needs equal partitions: ranks hold %d..%d samples" % (lo, hi))

    def size(self):
        return self.n * (self.world if self.presharded else 1)

    def num_of_slice(self):
        return self._slices

    def _order(self, train, epoch):
        if train and self.shuffle_:
            rng = np.random.default_rng(1234 + (epoch or 0) + (7919 * self.rank if self.presharded else 0))
            perm = rng.permutation(self.n)
        else:
            perm = np.arange(self.n)
        if self.world > 1 and not self.presharded:
            per = self.n // self.world if (train or self.drop_last) else int(math.ceil(self.n / self.world))
            shard = perm[self.rank::self.world][:per]
            return shard
        return perm

    def data(self, train=True, epoch=None):
        order = self._order(train, epoch)
        if self._slices > 1 and train:
            # sliced epoch: one 1/num_slice portion of the shuffled data per call
            k = (epoch or 0) % self._slices
            part = len(order) // self._slices
            order = order[k * part:(k + 1) * part]
        bs = self.local_bs
        nb = len(order) // bs if (train and self.drop_last) else int(math.ceil(len(order) / bs))
        if self._dev_arrays is not None:
            return self._iter_device(order, nb, bs)
        return self._iter_host(order, nb, bs)

    def _split(self, tensors):
        nx = len(self.xs)
        x = tensors[:nx]
        y = tensors[nx:]
        xo = x if self.multi_x else x[0]
        if self.ys is None:
            return (xo,)
        yo = y if self.multi_y else y[0]
        return (xo, yo)

    def _iter_device(self, order, nb, bs):
        dev = self._dev_arrays[0].device
        idx_all = torch.from_numpy(order.astype(np.int64)).to(dev)
        for b in range(nb):
            idx = idx_all[b * bs:(b + 1) * bs]
            yield self._split([a.index_select(0, idx) for a in self._dev_arrays])

    def _iter_host(self, order, nb, bs):
        g = _gatherer()
        pin = torch.cuda.is_available()
        srcs = self._pinned or [torch.from_numpy(a) for a in self.xs + (self.ys or [])]
        depth = 2
        pending = []

        def launch(b):
            idx = np.ascontiguousarray(order[b * bs:(b + 1) * bs].astype(np.int64))
            outs, tickets = [], []
            for s in srcs:
                o = torch.empty((len(idx),) + tuple(s.shape[1:]), dtype=s.dtype, pin_memory=pin)
                if g is not None and s.is_contiguous():
                    row = s[0].numel() * s.element_size() if s.dim() > 1 else s.element_size()
                    tickets.append(g.submit(s.data_ptr(), s.shape[0], row, idx.ctypes.data, len(idx), o.data_ptr()))
                else:
                    o.copy_(s[torch.from_numpy(idx)])
                outs.append(o)
            return outs, tickets, idx

        try:
            for b in range(min(depth, nb)):
                pending.append(launch(b))
            for b in range(nb):
                outs, tickets, _idx = pending.pop(0)
                for t in tickets:
                    g.wait(t)
                if b + depth < nb:
                    pending.append(launch(b + depth))
                yield self._split(outs)
        finally:
            # an abandoned epoch (exception / early break) must not free the
            # destination buffers and index arrays while gather workers still
            # write into / read from them
            for _outs, tickets, _idx in pending:
                for t in tickets:
                    g.wait(t)


class DataLoaderFeatureSet(FeatureSet):
    def __init__(self, loader):
        self.loader = loader

    def size(self):
        try:
            return len(self.loader.dataset)
        except Exception:  # noqa: BLE001
            return -1

    def data(self, train=True, epoch=None):
        sampler = getattr(self.loader, "sampler", None)
        if hasattr(sampler, "set_epoch") and epoch is not None:
            sampler.set_epoch(epoch)
        for b in self.loader:
            yield tuple(b) if isinstance(b, (list, tuple)) else (b,)


class GeneratorFeatureSet(FeatureSet):
    def __init__(self, fn, size=None):
        self.fn, self._size = fn, size

    def size(self):
        return self._size if self._size is not None else -1

    def data(self, train=True, epoch=None):
        for b in self.fn():
            yield tuple(b) if isinstance(b, (list, tuple)) else (b,)


class TransformedFeatureSet(FeatureSet):
    def __init__(self, base, preprocessing):
        self.base, self.pre = base, preprocessing

    def size(self):
        return self.base.size()

    def data(self, train=True, epoch=None):
        for b in self.base.data(train, epoch):
            yield self.pre(b)


# ----------------------------------------------------------------------------
# Preprocessing algebra (Zs/feature/common/Preprocessing.scala:35-82, ->)
# ----------------------------------------------------------------------------
class Preprocessing:
    """A composable record transform; ``a -> b`` is ``a >> b`` (or ChainedPreprocessing)."""

    def __call__(self, x):
        return self.apply(x)

    def apply(self, x):
        raise NotImplementedError

    def __rshift__(self, other):
        return ChainedPreprocessing([self, other])


class ChainedPreprocessing(Preprocessing):
    def __init__(self, transformers):
        self.transformers = []
        for t in transformers:
            if isinstance(t, ChainedPreprocessing):
                self.transformers.extend(t.transformers)
            else:
                self.transformers.append(t)

    def apply(self, x):
        for t in self.transformers:
            x = t(x)
        return x


class Lambda(Preprocessing):
    def __init__(self, fn):
        self.fn = fn

    def apply(self, x):
        return self.fn(x)


class ScalarToTensor(Preprocessing):
    def apply(self, x):
        return torch.tensor([float(x)])


class SeqToTensor(Preprocessing):
    def __init__(self, size=None):
        self.size = size

    def apply(self, x):
        t = torch.as_tensor(np.asarray(x, dtype=np.float32))
        return t.reshape(self.size) if self.size else t


class SeqToMultipleTensors(Preprocessing):
    def __init__(self, size):
        self.size = size

    def apply(self, x):
        arr = np.asarray(x, dtype=np.float32)
        out, off = [], 0
        for s in self.size:
            n = int(np.prod(s))
            out.append(torch.as_tensor(arr[off:off + n]).reshape(s))
            off += n
        return out


class ArrayToTensor(SeqToTensor):
    pass


class MLlibVectorToTensor(SeqToTensor):
    def apply(self, x):
        return super().apply(x.toArray() if hasattr(x, "toArray") else x)


class TensorToSample(Preprocessing):
    def apply(self, x):
        return (x,)


class FeatureLabelPreprocessing(Preprocessing):
    def __init__(self, feature_transformer, label_transformer):
        self.f, self.l = feature_transformer, label_transformer

    def apply(self, x):
        feat, label = x
        return (self.f(feat), self.l(label))


class MultiTensorsToSample(Preprocessing):
    def apply(self, x):
        return tuple(x)


class FeatureToTupleAdapter(Preprocessing):
    def __init__(self, sample_transformer):
        self.t = sample_transformer

    def apply(self, x):
        return self.t(x)


class ToTuple(Preprocessing):
    def apply(self, x):
        return tuple(x) if isinstance(x, (list, tuple)) else (x,)


class SampleToMiniBatch(Preprocessing):
    """Stack a list of samples (tuples of arrays) into one minibatch."""

    def __init__(self, batch_size=32, partition_num=None):
        self.batch_size = batch_size

    def apply(self, samples):
        cols = list(zip(*samples))
        return tuple(torch.as_tensor(np.stack([np.asarray(c) for c in col])) for col in cols)
