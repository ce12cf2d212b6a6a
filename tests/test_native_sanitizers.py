"""Builds the host-only native runtime pieces (thread pool, eigensolver, text readers) with
AddressSanitizer + UndefinedBehaviorSanitizer and, separately, ThreadSanitizer, and runs the
C++ unit tests in tests/native/test_native.cpp under each (CPU only; GPU sanitizers are not
available on the MI355X pool, per the task environment)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = "/opt/rocm/llvm/bin/clang++"
SRCS = ["csrc/runtime/thread_pool.cpp", "csrc/linalg/eigen.cpp", "csrc/io/text_reader.cpp",
        "tests/native/test_native.cpp"]


@pytest.mark.skipif(not os.path.exists(CXX), reason="ROCm clang++ not available")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_native_under_sanitizer(tmp_path, san):
    exe = tmp_path / "native_tests"
    cmd = [CXX, "-x", "c++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{ROOT}/csrc",
           f"-fsanitize={san}", "-fno-sanitize-recover=all", "-pthread"]
    cmd += [os.path.join(ROOT, s) for s in SRCS] + ["-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "native tests ok" in r.stdout
