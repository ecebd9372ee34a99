"""the CPU oracle (and the synthetic generator / host setup code it
runs with) is clean under AddressSanitizer + UndefinedBehaviorSanitizer over every test
camera, the ragged small case, the stage-by-stage entry points, the keyframe decision and
the numeric helpers (oracle/asan_driver.cpp, `make oracle-asan`)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan():
    if shutil.which("g++") is None or shutil.which("make") is None:
        pytest.skip("no host toolchain")
    r = subprocess.run(["make", "-s", "oracle-asan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "oracle sanitizer run: clean" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
