"""Py/util/engine.py: the reference locates SPARK_HOME / the zoo jars here. This
framework has no JVM side, so environment preparation reduces to the ROCm
process settings the engine needs (kept idempotent)."""
import os


def exist_pyspark():
    try:
        import pyspark  # noqa: F401
        return True
    except ImportError:
        return False


def prepare_env():
    # dmabuf IPC is the only mode the host driver supports for RCCL / tensor sharing
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def get_analytics_zoo_classpath():
    return ""


def compare_version(version1, version2):
    a = [int(x) for x in str(version1).split(".") if x.isdigit()]
    b = [int(x) for x in str(version2).split(".") if x.isdigit()]
    return (a > b) - (a < b)
