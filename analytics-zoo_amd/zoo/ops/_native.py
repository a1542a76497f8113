"""Loader for the in-tree HIP kernel library ``zoo._C``.

GPU tensors ALWAYS go through the native gfx950 kernels: if the extension is
missing on a machine with a GPU, the first op raises instead of silently
falling back to an eager PyTorch path. CPU tensors use the PyTorch reference
implementations in each op module (these double as the numerics oracles in
tests/).
"""
import importlib
import os

_C = None
_err = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        _C = importlib.import_module("zoo._C")
    except ImportError as e:  # pragma: no cover - depends on build state
        if os.environ.get("ZOO_AUTOBUILD", "1") == "1":
            try:
                from zoo.utils.build import build_native
                build_native()
                _C = importlib.import_module("zoo._C")
                return _C
            except Exception as e2:  # noqa: BLE001
                _err = e2
                return None
        _err = e
    return _C


def native():
    """Return the native module, raising loudly if it cannot be loaded."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "zoo native HIP library (zoo._C) is not available: %r. Build it with "
            "`python analytics-zoo_amd/tools/build_native.py`." % (_err,))
    return m


def available():
    return _load() is not None


def on_gpu(t):
    return t is not None and t.is_cuda


def set_deterministic(on=True):
    """Bit-reproducible reductions on the conv / BN / loss path:
    every cross-workgroup float sum goes through per-workgroup partials folded in
    a fixed order instead of fp32 atomics. Also set by ``ZOO_DETERMINISTIC=1``."""
    native().set_deterministic(bool(on))


def deterministic():
    m = _load()
    return bool(m.get_deterministic()) if m is not None else False


def native_build_info():
    """Provenance of the loaded native libraries: the manifest written by the build
    (tools/build_native.py) plus ``source_hash_matches`` -- whether that build was made from
    the csrc/ files present in this tree right now (content hashes, not mtimes)."""
    import json
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(pkg, "_build_manifest.json")
    info = {"manifest": None, "source_hash_matches": None, "loaded": available()}
    if os.path.exists(path):
        with open(path) as f:
            info["manifest"] = json.load(f)
        try:
            from zoo.utils.build import tree_source_hash
            cur = tree_source_hash()
            info["tree_source_hash"] = cur
            info["source_hash_matches"] = cur == info["manifest"].get("source_hash")
        except (OSError, ImportError):
            pass
    return info
