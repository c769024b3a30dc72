"""Host sanitizer builds (ASan + UBSan, every report fatal) of the CPU code that runs without a GPU
(tests/sanitize/Makefile): the oracle's whole path on C0 / non-dense + NaN / custom layout / rect
mode 1 / tiny / empty clouds, the synthetic generator, and the product's host Subdiv2D replay
(active-orchard-slam_amd/csrc/subdiv2d.cpp) under tools/sdcheck's per-insert state equivalence
checker (cavity insert vs OpenCV's swap loop). The GPU-side code cannot run here; GPU ASan is not
available on the test pool."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = "/tmp/aos_sanitize"


@pytest.fixture(scope="module")
def built():
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "sanitize"), f"OUT={OUT}"], check=True)
    return OUT


def _run(cmd, env=None, timeout=600):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, text=True, env=e, timeout=timeout)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    return r.stdout


def test_oracle_under_asan_ubsan(built):
    out = _run([os.path.join(built, "san_oracle")])
    assert "all frames ok" in out


def test_host_subdiv2d_under_asan_ubsan(built):
    out = _run([os.path.join(built, "san_sdcheck")], env={"AOS_SDCHECK_REPS": "2"})
    assert "0 failed so far" in out.splitlines()[-1]
