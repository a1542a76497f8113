"""Helpers of Py/common/utils.py (paths, remote files, JTensor/Sample) on the
native runtime — there is no JVM, so ``callZooFunc`` has nothing to call."""
import os
import tempfile
import uuid

import numpy as np

from zoo.utils.file import (get_remote_file_to_local, is_local_path,  # noqa: F401
                            put_local_file_to_remote)


def convert_to_safe_path(input_path, follow_symlinks=True):
    return os.path.realpath(input_path) if follow_symlinks else os.path.abspath(input_path)


def to_list_of_numpy(elements):
    if isinstance(elements, np.ndarray):
        return [elements]
    if np.isscalar(elements):
        return [np.array(elements)]
    if not isinstance(elements, list):
        raise ValueError("Wrong type: %s" % type(elements))
    out = []
    for e in elements:
        if np.isscalar(e):
            out.append(np.array(e))
        elif isinstance(e, np.ndarray):
            out.append(e)
        else:
            raise ValueError("Wrong type: %s" % type(e))
    return out


def append_suffix(prefix, path):
    ext = os.path.splitext(str(path))[1]
    return prefix + ext if ext else prefix


def _scratch_for(path):
    return os.path.join(tempfile.gettempdir(), append_suffix(str(uuid.uuid1()), path))


def save_file(save_func, path):
    """Run ``save_func(local_path)``; remote targets are written locally then uploaded."""
    if is_local_path(path):
        save_func(path)
        return
    tmp = _scratch_for(path)
    try:
        save_func(tmp)
        put_local_file_to_remote(tmp, path, over_write=True)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def load_from_file(load_func, path):
    if is_local_path(path):
        return load_func(path)
    tmp = _scratch_for(path)
    get_remote_file_to_local(path, tmp, over_write=True)
    try:
        return load_func(tmp)
    finally:
        os.remove(tmp)


def set_core_number(num):
    """PythonZoo.setCoreNumber: host threads for CPU ops / data loading."""
    import torch
    torch.set_num_threads(int(num))
    os.environ["ZOO_LOADER_THREADS"] = str(int(num))


def callZooFunc(bigdl_type, name, *args):  # noqa: N802 - reference name
    raise NotImplementedError("callZooFunc(%s): there is no JVM bridge; every zoo API is native Python here"
                              % name)


class JTensor:
    """numpy carrier with the reference's JTensor surface (storage/shape/indices)."""

    def __init__(self, storage, shape, bigdl_type="float", indices=None):
        self.storage = np.asarray(storage)
        self.shape = np.asarray(shape, dtype=np.int64)
        self.indices = None if indices is None else np.asarray(indices)
        self.bigdl_type = bigdl_type

    @classmethod
    def from_ndarray(cls, a_ndarray, bigdl_type="float"):
        a = np.asarray(a_ndarray)
        return cls(a.reshape(-1), a.shape, bigdl_type)

    @classmethod
    def sparse(cls, a_ndarray, i_ndarray, shape, bigdl_type="float"):
        return cls(np.asarray(a_ndarray), shape, bigdl_type, np.asarray(i_ndarray))

    def to_ndarray(self):
        if self.indices is not None:
            dense = np.zeros(tuple(self.shape), dtype=self.storage.dtype)
            idx = self.indices.reshape(len(self.shape), -1)
            dense[tuple(idx)] = self.storage
            return dense
        return self.storage.reshape(tuple(self.shape))

    def __repr__(self):
        return "JTensor(shape=%s)" % (tuple(self.shape),)


class Sample:
    """features + labels as lists of ndarrays (BigDL Sample)."""

    def __init__(self, features, labels, bigdl_type="float"):
        self.features = to_list_of_numpy(features if isinstance(features, list) else np.asarray(features))
        self.labels = to_list_of_numpy(labels if isinstance(labels, list) else np.asarray(labels))
        self.bigdl_type = bigdl_type

    @classmethod
    def from_ndarray(cls, features, labels, bigdl_type="float"):
        return cls(features, labels, bigdl_type)

    @property
    def feature(self):
        return self.features[0]

    @property
    def label(self):
        return self.labels[0]
