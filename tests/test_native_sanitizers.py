"""Race detection / memory-error checks for the native host runtime.

Builds tests/native/core_sanitize_test.cc (which #includes the `_pscore` sources
without their pybind layer) under ThreadSanitizer and under
AddressSanitizer+UndefinedBehaviorSanitizer, then runs each binary: it drives the
TCP Van, TaskTracker, text-proto parser, data parser and crc32c from many threads.
Host code only; no GPU.

ROCm's clang is used (its compiler-rt intercepts pthread_cond_clockwait, which
libstdc++'s condition_variable::wait_for calls; gcc 11's libtsan does not and
reports false "double lock" errors). Falls back to g++ for ASan if needed.
"""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "native" / "core_sanitize_test.cc"
INC = ROOT / "parameter_server_amd" / "csrc" / "core"
ROCM_CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def _compiler():
    if os.path.exists(ROCM_CLANG):
        return ROCM_CLANG
    return shutil.which("clang++")


def _build_and_run(tmp_path, flags, name):
    cxx = _compiler()
    if cxx is None:
        pytest.skip("no clang++ with sanitizer runtimes")
    exe = tmp_path / name
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-pthread", "-fno-omit-frame-pointer", *flags,
           f"-I{INC}", str(SRC), "-o", str(exe), "-lz"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1 verify_asan_link_order=0 halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1 halt_on_error=1"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "core_sanitize_test OK" in r.stdout
    for bad in ("ThreadSanitizer", "AddressSanitizer", "runtime error:", "LeakSanitizer"):
        assert bad not in out, out[-6000:]


def test_runtime_under_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], "core_tsan")


def test_runtime_under_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   "core_asan")
