#!/usr/bin/env python3
"""Build the zoo native libraries in-tree for MI355X (gfx950).

  zoo/_C*.so        HIP kernel library + torch bindings  (csrc/kernels/*.hip, csrc/ops.cpp)
  zoo/_runtime*.so  host C++ runtime (data loader, TFRecord/CRC32C writer,
                    protobuf wire codec, serving batch queue)  (csrc/runtime/*.cpp)

HIP sources are compiled directly with ``hipcc --offload-arch=gfx950`` (no
hipify, no CUDA shims); the binding layer is compiled with g++ against the
PyTorch-ROCm headers. Objects are rebuilt only when a source or header is
newer than the object, so repeated builds take a second.

Usage:  python analytics-zoo_amd/tools/build_native.py [--force] [-j N]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)                 # analytics-zoo_amd/
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "zoo")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("ZOO_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    return tdir, [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newer(src_list, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n%s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def build_kernels(force=False, jobs=8, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    tdir, tinc = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    objs, tasks = [], []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src] + headers, obj):
            tasks.append([HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
                          "-munsafe-fp-atomics", "-c", src, "-o", obj])
    bsrc = os.path.join(CSRC, "ops.cpp")
    bobj = os.path.join(BUILD, "ops.cpp.o")
    objs.append(bobj)
    if force or _newer([bsrc] + headers, bobj):
        tasks.append(["g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                      "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                      "-D_GLIBCXX_USE_CXX11_ABI=1"] + ["-I" + p for p in tinc] +
                     ["-I/opt/rocm/include", "-I" + pyinc, "-c", bsrc, "-o", bobj])
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(_run, tasks))
    out = os.path.join(PKG, "_C" + _ext_suffix())
    if force or tasks or not os.path.exists(out):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out] + objs +
             ["-L" + os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              "-ltorch_python", "-Wl,-rpath," + os.path.join(tdir, "lib")])
        if verbose:
            print("built", out)
    return out


def build_runtime(force=False, jobs=8, verbose=True):
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return None
    os.makedirs(BUILD, exist_ok=True)
    import pybind11
    pyinc = sysconfig.get_paths()["include"]
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    objs, tasks = [], []
    for src in srcs:
        obj = os.path.join(BUILD, "rt_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src] + headers, obj):
            tasks.append(["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", "-I" + pybind11.get_include(),
                          "-I" + pyinc, "-c", src, "-o", obj])
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(_run, tasks))
    out = os.path.join(PKG, "_runtime" + _ext_suffix())
    if force or tasks or not os.path.exists(out):
        _run(["g++", "-shared", "-fPIC", "-pthread", "-o", out] + objs)
        if verbose:
            print("built", out)
    return out


def build_all(force=False, jobs=8, verbose=True):
    build_kernels(force, jobs, verbose)
    build_runtime(force, jobs, verbose)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    try:
        build_all(a.force, a.j)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
