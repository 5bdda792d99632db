"""Host-side AddressSanitizer + UBSan run of the C ABI (CPU; no GPU needed).

libhdgnn's host code (argument validation, shape / path resolution, sizing, layouts, error
reporting, the device entry points up to their first device call) is rebuilt with
`-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined` (GPU code untouched:
device sanitizers are not available on this pool) into a scratch directory, linked to the
clang-built, sanitized driver tests/host/asan_abi.c, and run; any sanitizer report or
failed check fails the test.  Skipped when the ROCm toolchain is absent.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/lib/llvm/bin/clang"


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)),
                    reason="ROCm toolchain absent")
@pytest.mark.timeout(900)
def test_abi_host_asan_ubsan(tmp_path):
    csrc = os.path.join(ROOT, "hd-gnn_amd", "csrc")
    inc = os.path.join(ROOT, "include")
    lib = tmp_path / "libhdgnn_asan.so"
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-g"]
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-fPIC", "-shared",
                    "-I" + inc] + san + ["-o", str(lib), os.path.join(csrc, "hdgnn.hip"),
                                         os.path.join(csrc, "wide.hip")],
                   check=True, timeout=800)
    exe = tmp_path / "asan_abi"
    subprocess.run([CLANG, "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-I" + inc, os.path.join(ROOT, "tests", "host", "asan_abi.c"), "-o", str(exe),
                    "-L" + str(tmp_path), "-lhdgnn_asan", "-Wl,-rpath," + str(tmp_path),
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"],
                   check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "all checks passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
