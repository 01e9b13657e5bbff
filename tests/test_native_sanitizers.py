"""The C++ P2P plane under AddressSanitizer + UndefinedBehaviorSanitizer.

csrc/net/selftest.cpp drives known-answer vectors, AEAD / Noise / secretstream fuzzing with tampering
and truncation, and a loopback transport session with an injected malformed frame.  Host code only:
GPU sanitizers are neither needed nor available for it."""
import os
import shutil
import subprocess

import pytest

from symmetry_amd import _build


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libubsan")
def test_net_plane_is_clean_under_asan_ubsan():
    exe = _build.build_selftest()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "net selftest: OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
