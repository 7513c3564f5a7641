"""The oracle and the CPU baseline under AddressSanitizer + UBSan (sanitizers on host
code): oracle/asan_driver.cpp runs every oracle entry point and cpu_baseline.cpp over seeded edge
shapes and round trips; any sanitizer report aborts it (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_oracle_and_cpu_baseline_clean_under_asan_ubsan():
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    out = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan-run"], capture_output=True,
                         text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "0 check failures" in out.stdout
