"""Checkpoint object IO.

Objects (state dicts of tensors, numbers, strings, lists, dicts) are written
with ``torch.save`` and read back with ``torch.load(weights_only=True)`` so
loading a checkpoint never executes code from the file. Paths may be local,
``file://`` or (through zoo.utils.file) ``hdfs://`` URIs; writes are atomic (temp file + rename) so a crash never
leaves a torn ``model.<n>`` that the failure-retry path would pick up.
"""
import os
import tempfile

import torch


def _local(path):
    if path.startswith("file://"):
        return path[len("file://"):]
    return path


def save_object(obj, path, overwrite=True):
    if "://" in path and not path.startswith("file://"):  # hdfs:// etc.: write locally, then upload
        from zoo.common.utils import save_file
        return save_file(lambda p: save_object(obj, p, True), path)
    path = _local(path)
    if os.path.exists(path) and not overwrite:
        raise FileExistsError(path)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix="zoo_tmp_", suffix=".part")
    os.close(fd)
    try:
        torch.save(obj, tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def save_bytes(data, path, overwrite=True):
    """Atomic write of raw bytes (same path rules as :func:`save_object`)."""
    if "://" in path and not path.startswith("file://"):
        from zoo.common.utils import save_file
        return save_file(lambda p: save_bytes(data, p, True), path)
    path = _local(path)
    if os.path.exists(path) and not overwrite:
        raise FileExistsError(path)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix="zoo_tmp_", suffix=".part")
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def load_object(path):
    if "://" in path and not path.startswith("file://"):
        from zoo.common.utils import load_from_file
        return load_from_file(load_object, path)
    return torch.load(_local(path), map_location="cpu", weights_only=True)
