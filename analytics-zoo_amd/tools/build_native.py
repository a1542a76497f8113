#!/usr/bin/env python3
"""Build the zoo native libraries in-tree for MI355X (gfx950).

  zoo/_C*.so        HIP kernel library + torch bindings  (csrc/kernels/*.hip, csrc/ops.cpp)
  zoo/_runtime*.so  host C++ runtime (data loader, TFRecord/CRC32C writer,
                    protobuf wire codec, serving batch queue)  (csrc/runtime/*.cpp)

HIP sources are compiled directly with ``hipcc --offload-arch=gfx950`` (no
hipify, no CUDA shims); the binding layer is compiled with g++ against the
PyTorch-ROCm headers.

Provenance: every object carries a ``.stamp`` = SHA-256 of (its source, every header it can
include, the exact compile command); an object is rebuilt when its stamp differs -- never on
file mtimes, which a snapshot / checkout does not preserve. Each library gets a manifest
(``zoo/_build_manifest.json``: the combined source hash, per-file hashes, the toolchain, the
time) and ``zoo.native_build_info()`` reports whether the loaded library was built from the
sources in the tree (``source_hash_matches``).

Usage:  python analytics-zoo_amd/tools/build_native.py [--force] [-j N] [--out DIR]
        (--out: clean out-of-tree build into DIR/{obj,zoo}, used by tests/test_build_provenance.py)
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
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
MANIFEST = "_build_manifest.json"


def _sha(paths, extra=""):
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(os.path.relpath(p, ROOT).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(extra.encode())
    return h.hexdigest()


def source_files():
    """Every file a native build reads from the tree."""
    pats = ["kernels/*.hip", "kernels/*.h", "ops.cpp", "comm.cpp", "runtime/*.cpp", "runtime/*.h"]
    out = []
    for pat in pats:
        out += glob.glob(os.path.join(CSRC, pat))
    return sorted(out)


def tree_source_hash():
    return _sha(source_files())


def _stale(obj, stamp):
    sp = obj + ".stamp"
    if not os.path.exists(obj) or not os.path.exists(sp):
        return True
    with open(sp) as f:
        return f.read().strip() != stamp


def _write_stamp(obj, stamp):
    with open(obj + ".stamp", "w") as f:
        f.write(stamp + "\n")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    return tdir, [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n%s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def _compile_all(jobs, items):
    """items: [(obj, stamp, cmd)] still to build -> run, then stamp each object."""
    def one(it):
        obj, stamp, cmd = it
        _run(cmd)
        _write_stamp(obj, stamp)
    if items:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(one, items))


def build_kernels(force=False, jobs=8, verbose=True, build_dir=None, pkg_dir=None):
    build_dir = build_dir or BUILD
    pkg_dir = pkg_dir or PKG
    os.makedirs(build_dir, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    tdir, tinc = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    objs, todo, stamps = [], [], []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-c", src,
               "-o", obj]
        stamp = _sha([src] + headers, " ".join(cmd[:-3]))
        objs.append(obj)
        stamps.append(stamp)
        if force or _stale(obj, stamp):
            todo.append((obj, stamp, cmd))
    bsrc = os.path.join(CSRC, "ops.cpp")
    bobj = os.path.join(build_dir, "ops.cpp.o")
    bcmd = ["g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
            "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-D_GLIBCXX_USE_CXX11_ABI=1"] + ["-I" + p for p in tinc] + \
        ["-I/opt/rocm/include", "-I" + pyinc, "-c", bsrc, "-o", bobj]
    bstamp = _sha([bsrc] + headers, " ".join(bcmd[:-3]))
    objs.append(bobj)
    stamps.append(bstamp)
    if force or _stale(bobj, bstamp):
        todo.append((bobj, bstamp, bcmd))
    # C++ comm layer (RCCL driven directly; the symbols resolve to torch's own librccl)
    csrc = os.path.join(CSRC, "comm.cpp")
    cobj = os.path.join(build_dir, "comm.cpp.o")
    ccmd = bcmd[:-3] + ["-c", csrc, "-o", cobj]
    cstamp = _sha([csrc], " ".join(ccmd[:-3]))
    objs.append(cobj)
    stamps.append(cstamp)
    if force or _stale(cobj, cstamp):
        todo.append((cobj, cstamp, ccmd))
    _compile_all(jobs, todo)
    out = os.path.join(pkg_dir, "_C" + _ext_suffix())
    link = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out] + objs + \
        ["-L" + os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
         "-ltorch_python", "-lrccl", "-Wl,-rpath," + os.path.join(tdir, "lib")]
    lstamp = hashlib.sha256(("".join(stamps) + " ".join(link[5:6])).encode()).hexdigest()
    if force or todo or _stale(out, lstamp):
        _run(link)
        _write_stamp(out, lstamp)
        if verbose:
            print("built", out)
    return out, len(todo)


def build_runtime(force=False, jobs=8, verbose=True, build_dir=None, pkg_dir=None):
    build_dir = build_dir or BUILD
    pkg_dir = pkg_dir or PKG
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return None, 0
    os.makedirs(build_dir, exist_ok=True)
    import pybind11
    pyinc = sysconfig.get_paths()["include"]
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    objs, todo, stamps = [], [], []
    for src in srcs:
        obj = os.path.join(build_dir, "rt_" + os.path.basename(src) + ".o")
        cmd = ["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", "-I" + pybind11.get_include(), "-I" + pyinc, "-c",
               src, "-o", obj]
        stamp = _sha([src] + headers, " ".join(cmd[:6]))
        objs.append(obj)
        stamps.append(stamp)
        if force or _stale(obj, stamp):
            todo.append((obj, stamp, cmd))
    _compile_all(jobs, todo)
    out = os.path.join(pkg_dir, "_runtime" + _ext_suffix())
    lstamp = hashlib.sha256("".join(stamps).encode()).hexdigest()
    if force or todo or _stale(out, lstamp):
        _run(["g++", "-shared", "-fPIC", "-pthread", "-o", out] + objs)
        _write_stamp(out, lstamp)
        if verbose:
            print("built", out)
    return out, len(todo)


def _toolchain():
    def ver(cmd):
        try:
            return subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                  timeout=60).stdout.strip().splitlines()[0]
        except (OSError, IndexError, subprocess.SubprocessError):
            return None
    return {"hipcc": ver([HIPCC, "--version"]), "gxx": ver(["g++", "--version"]), "arch": ARCH}


def build_all(force=False, jobs=8, verbose=True, out_dir=None):
    """Build both libraries (in-tree, or clean into ``out_dir``/{obj,zoo}) and write the
    provenance manifest next to them. Returns the manifest dict."""
    import time
    build_dir = os.path.join(out_dir, "obj") if out_dir else None
    pkg_dir = os.path.join(out_dir, "zoo") if out_dir else None
    if pkg_dir:
        os.makedirs(pkg_dir, exist_ok=True)
    c_so, c_n = build_kernels(force, jobs, verbose, build_dir, pkg_dir)
    r_so, r_n = build_runtime(force, jobs, verbose, build_dir, pkg_dir)
    man = {"source_hash": tree_source_hash(),
           "files": {os.path.relpath(p, ROOT): _sha([p]) for p in source_files()},
           "libraries": {os.path.basename(p): open(p + ".stamp").read().strip() for p in (c_so, r_so) if p},
           "objects_compiled": c_n + r_n, "forced": bool(force), "toolchain": _toolchain(),
           "built_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    with open(os.path.join(pkg_dir or PKG, MANIFEST), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    return man


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--out", default=None, help="clean out-of-tree build directory")
    a = ap.parse_args()
    try:
        m = build_all(a.force, a.j, out_dir=a.out)
        print("source_hash", m["source_hash"], "objects_compiled", m["objects_compiled"])
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
