"""Host build under AddressSanitizer + UndefinedBehaviorSanitizer: the C API
stress driver (tests/c/api_stress.c) must run clean (GPU
sanitizers are not available, so the sanitized build is the host one)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc with libasan")
def test_asan_ubsan_api_stress():
    out = subprocess.run(["make", "-C", ROOT, "asan-check"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-5000:]
    assert "checkpoint ok" in out.stdout
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
