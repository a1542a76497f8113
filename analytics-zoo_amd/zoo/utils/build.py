"""Programmatic access to the native build (used by __graft_entry__.build and autobuild)."""
import importlib.util
import os

_TOOLS = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools",
                      "build_native.py")


def _mod():
    spec = importlib.util.spec_from_file_location("zoo_build_native", _TOOLS)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def build_native(force=False, jobs=8, verbose=False, out_dir=None):
    """Content-stamped build (rebuilds exactly the objects whose source / headers / command
    changed); returns the provenance manifest."""
    return _mod().build_all(force=force, jobs=jobs, verbose=verbose, out_dir=out_dir)


def tree_source_hash():
    return _mod().tree_source_hash()
