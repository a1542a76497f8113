"""Host-runtime sanitizer builds: the serving queue / RESP server,
Gatherer, CRC32C/TFRecord and protobuf scanner compiled with ASan+UBSan and with TSan
(tools/sanitize_runtime.py, Python bindings compiled out) must run their self-test
without a report. CPU only."""
import importlib.util
import os
import shutil

import pytest

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "analytics-zoo_amd")


def _tool():
    spec = importlib.util.spec_from_file_location("sanitize_runtime", os.path.join(ROOT, "tools", "sanitize_runtime.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.skipif(shutil.which("g++") is None and not os.path.exists("/opt/rocm/lib/llvm/bin/clang++"),
                    reason="no host C++ compiler")
@pytest.mark.parametrize("config", ["asan", "tsan"])
def test_runtime_selftest_under_sanitizer(config):
    code, out = _tool().run(config)
    assert code == 0 and "rt_selftest: PASSED" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "runtime error:" not in out  # UBSan
