"""Py/util/engine.py: the reference locates SPARK_HOME / the zoo jars and prepares the
Spark environment here (``prepare_env``, ``get_analytics_zoo_classpath``,
``check_spark_source_conflict``). This framework has no JVM side; its environment is the
ROCm runtime and the process layout of a one-process-per-GPU job, so ``prepare_env``
sets the HIP/RCCL process settings (idempotently, never overriding user values) and
``get_env_info`` reports what the engine will run on.
"""
import os
import platform
import shutil


def exist_pyspark():
    try:
        import pyspark  # noqa: F401
        return True
    except ImportError:
        return False


def rocm_path():
    return os.environ.get("ROCM_PATH") or ("/opt/rocm" if os.path.isdir("/opt/rocm") else None)


def rocm_version():
    p = rocm_path()
    if not p:
        return None
    for f in (os.path.join(p, ".info", "version"), os.path.join(p, ".info", "version-dev")):
        if os.path.exists(f):
            with open(f) as fh:
                return fh.read().strip()
    return None


def prepare_env(local_world_size=None):
    """Process settings for a rank of a zoo job:

    * ``HSA_ENABLE_IPC_MODE_LEGACY=0``: dmabuf IPC, the only mode the host driver offers for
      RCCL and cross-process tensor sharing;
    * ``OMP_NUM_THREADS``: the node's CPUs split over the local ranks (data loading and
      host-side ops of one rank must not oversubscribe the others);
    * ``ZOO_NATIVE_LIB``: the in-tree kernel library's directory, for tools that load it
      without importing the package.
    """
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    n = int(local_world_size or os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    os.environ.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // max(n, 1))))
    os.environ.setdefault("ZOO_NATIVE_LIB", os.path.join(os.path.dirname(os.path.dirname(__file__))))
    return dict((k, os.environ[k]) for k in ("HSA_ENABLE_IPC_MODE_LEGACY", "OMP_NUM_THREADS", "ZOO_NATIVE_LIB"))


def get_env_info():
    """What the engine runs on: Python, torch/HIP, ROCm install, visible GPUs, native library."""
    info = {"python": platform.python_version(), "platform": platform.platform(), "rocm_path": rocm_path(),
            "rocm_version": rocm_version(), "hipcc": shutil.which("hipcc") or (
                os.path.join(rocm_path(), "bin", "hipcc") if rocm_path() else None)}
    try:
        import torch
        info.update(torch=torch.__version__, hip=getattr(torch.version, "hip", None),
                    gpus=torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        info.update(torch=None, hip=None, gpus=0)
    try:
        from zoo.ops._native import available
        info["native_kernels"] = bool(available())
    except Exception:  # noqa: BLE001
        info["native_kernels"] = False
    return info


def get_analytics_zoo_classpath():
    """No JVM classpath: the native libraries are in-tree (``zoo/_C*.so``, ``zoo/_runtime*.so``)."""
    return ""


def is_spark_below_2_2():
    return False


def check_spark_source_conflict(spark_home=None, pyspark_path=None):
    return None


def compare_version(version1, version2):
    a = [int(x) for x in str(version1).split(".") if x.isdigit()]
    b = [int(x) for x in str(version2).split(".") if x.isdigit()]
    return (a > b) - (a < b)
