"""Sanitizer runs of the C-ABI's host code: ``build.py --asan`` / ``--tsan`` build
``csrc/lsa.cpp`` + ``csrc/sparse_host.cpp`` with AddressSanitizer + UBSan / ThreadSanitizer and link
the driver ``tests/asan/host_driver.cpp`` (LSAP pool on random / tie / rectangular / padded batches
against brute force and the single-thread result; the sparse host twins against dense products).
The ASan driver runs once per LSA solver path.  CPU only (GPU sanitizers are unavailable)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fingerprint-matching-code_amd"))

pytestmark = pytest.mark.skipif(shutil.which(os.environ.get("CXX", "g++")) is None, reason="no host C++ compiler")


def _run(binary, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:exitcode=23"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=66"
    r = subprocess.run([binary], env=env, capture_output=True, text=True, timeout=600)
    bad = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")
    assert r.returncode == 0 and not any(b in r.stderr for b in bad), (r.returncode, r.stderr[-4000:])
    assert "all checks passed" in r.stdout


@pytest.mark.parametrize("path", ["", "FPM_LSA_SCALAR", "FPM_LSA_AVX2", "FPM_LSA_DENSE512"])
def test_host_code_under_asan(path):
    import build
    binary = build.build_asan(verbose=False, kind="asan")
    _run(binary, {path: "1"} if path else {})


def test_lsa_pool_under_tsan():
    import build
    binary = build.build_asan(verbose=False, kind="tsan")
    _run(binary, {})
