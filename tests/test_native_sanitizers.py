"""Host-code sanitizer tier: the C++ contour oracle built with
AddressSanitizer + UndefinedBehaviorSanitizer and run over random label maps.
(GPU sanitizers are not available on the MI355X pool; device code is covered by
the kernel goldens and the stream-ordered, capture-checked graph tests.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_contour_oracle_under_asan_ubsan(tmp_path):
    exe = tmp_path / "contours_selftest"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I", os.path.join(ROOT, "csrc", "host"),
           os.path.join(ROOT, "tests", "native", "contours_selftest.cpp"),
           os.path.join(ROOT, "csrc", "host", "contours.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload other libraries ahead
    # of the ASan runtime; they are left as they are
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "300"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ok 300 maps" in r.stdout
