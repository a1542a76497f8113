"""Build provenance: a CLEAN out-of-tree build of both native libraries
from the sources in this checkout compiles every object, records the source hash it was built
from, loads, and an unchanged re-build compiles nothing -- even after file mtimes change (the
stamps are content hashes, so a stale prebuilt library cannot pass for a fresh one)."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "analytics-zoo_amd")
TOOL = os.path.join(PKG, "tools", "build_native.py")


def _tool():
    spec = importlib.util.spec_from_file_location("zoo_build_native_t", TOOL)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_clean_out_of_tree_build_is_stamped_and_loads(tmp_path):
    out = str(tmp_path / "build")
    r = subprocess.run([sys.executable, TOOL, "--force", "-j", "8", "--out", out], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=1500)
    assert r.returncode == 0, r.stdout[-3000:]
    tool = _tool()
    with open(os.path.join(out, "zoo", "_build_manifest.json")) as f:
        man = json.load(f)
    assert man["source_hash"] == tool.tree_source_hash()
    n_src = len([p for p in tool.source_files() if p.endswith((".hip", ".cpp"))])
    assert man["objects_compiled"] == n_src and man["forced"]
    assert man["toolchain"]["arch"] == "gfx950"
    libs = sorted(os.listdir(os.path.join(out, "zoo")))
    assert any(l.startswith("_C") and l.endswith(".so") for l in libs)
    assert any(l.startswith("_runtime") and l.endswith(".so") for l in libs)
    # the fresh library loads and answers (in a child: it must not clash with the in-tree zoo._C)
    so = [os.path.join(out, "zoo", l) for l in libs if l.startswith("_C") and l.endswith(".so")][0]
    code = ("import importlib.util,torch;s=importlib.util.spec_from_file_location('zoo._C',%r);"
            "m=importlib.util.module_from_spec(s);s.loader.exec_module(m);print(m.stat_len(64))" % so)
    c = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300)
    assert c.returncode == 0 and int(c.stdout.strip().splitlines()[-1]) >= 128, c.stdout[-2000:]
    # unchanged sources: nothing recompiles, whatever the mtimes say
    for p in tool.source_files()[:3]:
        os.utime(p, None)
    r2 = subprocess.run([sys.executable, TOOL, "-j", "8", "--out", out], stdout=subprocess.PIPE,
                        stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r2.returncode == 0, r2.stdout[-2000:]
    assert "objects_compiled 0" in r2.stdout


def test_stamp_changes_with_content_not_mtime(tmp_path):
    tool = _tool()
    a = tmp_path / "a.hip"
    a.write_text("int x = 1;\n")
    s1 = tool._sha([str(a)], "cmd")
    os.utime(a, (1, 1))
    assert tool._sha([str(a)], "cmd") == s1
    a.write_text("int x = 2;\n")
    assert tool._sha([str(a)], "cmd") != s1
    assert tool._sha([str(a)], "cmd -O2") != tool._sha([str(a)], "cmd -O3")
