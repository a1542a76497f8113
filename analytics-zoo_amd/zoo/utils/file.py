"""File-system helpers (Zs/common/Utils.scala:35-278 FS helpers; Zs/utils/File.scala:24-112
FileReader/FileWriter over Hadoop FS).

Paths may be plain local paths, ``file://`` URIs, ``hdfs://`` URIs or ``s3://``
(``s3a://``, ``s3n://``) URIs. Local paths go through the OS directly; ``hdfs://``
goes through the ``hdfs dfs`` CLI when one is on PATH (there is no JVM/Hadoop client
in this framework); ``s3://`` goes through the built-in SigV4 client
(``zoo.utils.s3``). Together they cover the copy-in / copy-out pattern the reference
uses for checkpoints and model files. Other schemes raise a clear error.
"""
import os
import shutil
import subprocess
import tempfile
import time
import uuid
from contextlib import contextmanager
from urllib.parse import urlparse


def scheme(path):
    return urlparse(str(path)).scheme.lower()


def is_local_path(path):
    return scheme(path) in ("", "file") or (len(scheme(path)) == 1 and os.name == "nt")


def local_path(path):
    """``file:///a/b`` -> ``/a/b``; plain paths unchanged."""
    p = str(path)
    return urlparse(p).path if scheme(p) == "file" else p


def _hdfs(*args, check=True):
    exe = shutil.which("hdfs")
    if exe is None:
        raise NotImplementedError("hdfs:// paths need the `hdfs` CLI on PATH (no Hadoop client in-process)")
    return subprocess.run([exe, "dfs"] + list(args), check=check, capture_output=True, text=True)


def _remote_only(path):
    if scheme(path) != "hdfs":
        raise NotImplementedError("unsupported file system scheme %r in %s" % (scheme(path), path))


def is_s3(path):
    return scheme(path) in ("s3", "s3a", "s3n")


def _s3():
    from zoo.utils import s3
    return s3.client(), s3.split_s3


def exists(path):
    if is_local_path(path):
        return os.path.exists(local_path(path))
    if is_s3(path):
        c, split = _s3()
        b, k = split(path)
        if k and c.head(b, k) is not None:
            return True
        keys, pre = c.list(b, k.rstrip("/") + "/" if k else "", "/")
        return bool(keys or pre)
    _remote_only(path)
    return _hdfs("-test", "-e", str(path), check=False).returncode == 0


def mkdirs(path):
    if is_local_path(path):
        os.makedirs(local_path(path), exist_ok=True)
        return
    if is_s3(path):   # object stores have no directories
        return
    _remote_only(path)
    _hdfs("-mkdir", "-p", str(path))


def list_files(path):
    if is_local_path(path):
        p = local_path(path)
        return sorted(os.path.join(p, f) for f in os.listdir(p)) if os.path.isdir(p) else [p]
    if is_s3(path):
        c, split = _s3()
        b, k = split(path)
        sch = scheme(path)
        if k and c.head(b, k) is not None:
            return [str(path)]
        keys, pre = c.list(b, k.rstrip("/") + "/" if k else "", "/")
        return sorted("%s://%s/%s" % (sch, b, x.rstrip("/")) for x in keys + pre)
    _remote_only(path)
    out = _hdfs("-ls", "-C", str(path)).stdout
    return sorted(line.strip() for line in out.splitlines() if line.strip())


def delete(path, recursive=True):
    if is_local_path(path):
        p = local_path(path)
        if os.path.isdir(p):
            shutil.rmtree(p) if recursive else os.rmdir(p)
        elif os.path.exists(p):
            os.remove(p)
        return
    if is_s3(path):
        c, split = _s3()
        b, k = split(path)
        c.delete(b, k)
        if recursive:
            for key in c.list(b, k.rstrip("/") + "/")[0]:
                c.delete(b, key)
        return
    _remote_only(path)
    _hdfs("-rm", "-f", "-r" if recursive else "", str(path))


def get_remote_file_to_local(remote_path, local, over_write=False):
    if not over_write and os.path.exists(local):
        raise FileExistsError(local)
    if is_local_path(remote_path):
        shutil.copyfile(local_path(remote_path), local)
        return
    if is_s3(remote_path):
        c, split = _s3()
        data = c.get(*split(remote_path))
        with open(local, "wb") as f:
            f.write(data)
        return
    _remote_only(remote_path)
    _hdfs("-get", "-f" if over_write else "", str(remote_path), local)


def put_local_file_to_remote(local, remote_path, over_write=False):
    if is_local_path(remote_path):
        dst = local_path(remote_path)
        if not over_write and os.path.exists(dst):
            raise FileExistsError(dst)
        d = os.path.dirname(os.path.abspath(dst))
        os.makedirs(d, exist_ok=True)
        shutil.copyfile(local, dst)
        return
    if is_s3(remote_path):
        c, split = _s3()
        b, k = split(remote_path)
        if not over_write and c.head(b, k) is not None:
            raise FileExistsError(str(remote_path))
        with open(local, "rb") as f:
            c.put(b, k, f.read())
        return
    _remote_only(remote_path)
    _hdfs("-put", "-f" if over_write else "", local, str(remote_path))


def read_bytes(path):
    with open_read(path) as f:
        return f.read()


def save_bytes(data, path, overwrite=False):
    with open_write(path, overwrite) as f:
        f.write(data)


@contextmanager
def open_read(path):
    """FileReader.open(): a binary stream for any supported path."""
    if is_local_path(path):
        with open(local_path(path), "rb") as f:
            yield f
        return
    tmp = os.path.join(tempfile.gettempdir(), "zoo_%s" % uuid.uuid4().hex)
    get_remote_file_to_local(path, tmp, over_write=True)
    try:
        with open(tmp, "rb") as f:
            yield f
    finally:
        os.remove(tmp)


@contextmanager
def open_write(path, overwrite=False):
    """FileWriter.create(overwrite): local writes are atomic (temp + rename)."""
    if is_local_path(path):
        dst = local_path(path)
        if not overwrite and os.path.exists(dst):
            raise FileExistsError(dst)
        d = os.path.dirname(os.path.abspath(dst))
        os.makedirs(d, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=d, prefix=".zoo_tmp_")
        try:
            with os.fdopen(fd, "wb") as f:
                yield f
            os.replace(tmp, dst)
        finally:
            if os.path.exists(tmp):
                os.remove(tmp)
        return
    tmp = os.path.join(tempfile.gettempdir(), "zoo_%s" % uuid.uuid4().hex)
    try:
        with open(tmp, "wb") as f:
            yield f
        put_local_file_to_remote(tmp, path, over_write=overwrite)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def create_tmp_dir(prefix="zoo"):
    """Utils.createTmpDir: a fresh local scratch directory."""
    return tempfile.mkdtemp(prefix=prefix + "_")


def time_it(name, logger=None):
    """Utils.timeIt as a context manager: logs the wall time of the block."""
    @contextmanager
    def _cm():
        t0 = time.perf_counter()
        yield
        msg = "%s time elapsed [%.3f s]" % (name, time.perf_counter() - t0)
        (logger.info if logger else print)(msg)
    return _cm()
