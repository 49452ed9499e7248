"""SURVEY.md §5 "Race detection / sanitizers": the C-ABI's host-side argument checks under AddressSanitizer.
tools/asan_build.sh compiles every csrc .hip source with -Xarch_host -fsanitize=address (device code unsanitized,
-O0: nothing under test reaches the GPU) and links tests/asan/capi_errors.c against it; the driver feeds invalid
descriptors to the descriptor-taking entry points and runs the pure host helpers to completion. Any ASan report
aborts the process."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/llvm/bin/clang++") or shutil.which("bash") is None,
                    reason="needs the ROCm clang toolchain")
def test_capi_error_paths_under_asan():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_build.sh"), "run"], capture_output=True, text=True,
                       timeout=900, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "PASSED: 0 failure(s)" in out and "ERROR: AddressSanitizer" not in out
