"""Sanitizer builds of the native host runtime.

Compiles csrc/runtime/selftest/rt_selftest.cpp -- which includes the host runtime sources
(serving queue + RESP front end, Gatherer, CRC32C/TFRecord, protobuf scanner) with the
Python bindings compiled out -- once per sanitizer configuration and runs it:

  asan : AddressSanitizer + UndefinedBehaviorSanitizer (heap/stack overflows, use-after-free,
         leaks, signed overflow, misaligned loads, bad shifts), aborting on the first report
  tsan : ThreadSanitizer (data races between the serving threads, worker pools, TCP
         connections and the shared CRC table)

The reference's equivalent is the JVM's memory safety plus Spark's task isolation; the
framework's host runtime is C++, so it gets compiler sanitizers instead. Host code only:
no GPU code is built here (GPU sanitizers are not available on the MI355X pool).

    python tools/sanitize_runtime.py            # both configurations
    python tools/sanitize_runtime.py asan       # one
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "runtime", "selftest", "rt_selftest.cpp")
OUT = os.path.join(ROOT, "build", "sanitize")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

CONFIGS = {
    "asan": (["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
             {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1:detect_stack_use_after_return=1",
              "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    "tsan": (["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
}


def build(name, cxx=None):
    flags, _ = CONFIGS[name]
    # ROCm's clang: its sanitizer runtimes intercept pthread_cond_clockwait, which the
    # system GCC 11 libtsan does not (false "double lock" reports on timed waits)
    cxx = cxx or os.environ.get("ZOO_SAN_CXX") or (CLANG if os.path.exists(CLANG) else "g++")
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "rt_selftest_" + name)
    deps = [SRC] + [os.path.join(ROOT, "csrc", "runtime", f) for f in ("runtime.cpp", "serving.cpp")]
    if not os.path.exists(exe) or any(os.path.getmtime(d) > os.path.getmtime(exe) for d in deps):
        cmd = [cxx, "-std=c++17", "-O1", "-g", "-pthread", "-Wall", "-Wextra", "-Wno-unused-function"] + flags + \
              [SRC, "-o", exe]
        subprocess.run(cmd, check=True)
    return exe


def run(name, timeout=300):
    exe = build(name)
    env = dict(os.environ)
    env.update(CONFIGS[name][1])
    p = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def main(argv):
    names = argv or list(CONFIGS)
    rc = 0
    for n in names:
        code, out = run(n)
        print("== %s (exit %d)\n%s" % (n, code, out.strip()))
        rc |= code != 0
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
