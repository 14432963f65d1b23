"""Native C++ host unit tests (bin/psoup_unit_tests) and their host
sanitizer builds (ASan/UBSan/TSan on the host code; GPU ASan
and XNACK are not available on the MI355X pool)."""
import os
import subprocess

import pytest

from conftest import REPO


def _run(exe):
    r = subprocess.run([exe, REPO], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout
    return r


def test_native_unit_tests():
    exe = os.path.join(REPO, "bin", "psoup_unit_tests")
    if not os.path.exists(exe):
        pytest.skip("native build missing (python peasoup_amd/_build.py)")
    _run(exe)


@pytest.mark.parametrize("san", ["address", "undefined", "thread"])
def test_native_unit_tests_under_host_sanitizers(san):
    from peasoup_amd import _build

    _build.build(sanitize=san)
    r = _run(os.path.join(REPO, "bin", f"psoup_unit_tests_{san}"))
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr


def test_thread_sanitizer_sees_an_injected_scheduler_race():
    """The TSan build runs the native scheduler's protocol clean (above); with
    the hand-over's lock removed (--inject-race) it must report the race, so a
    clean run is evidence, not an unobserved path."""
    from peasoup_amd import _build

    _build.build(sanitize="thread")
    exe = os.path.join(REPO, "bin", "psoup_unit_tests_thread")
    r = subprocess.run([exe, "--inject-race"], capture_output=True, text=True, timeout=300)
    assert "WARNING: ThreadSanitizer: data race" in r.stderr, r.stderr[-3000:]
    assert "ChunkScheduler" in r.stderr and "finalize" in r.stderr
