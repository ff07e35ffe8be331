"""The native relay (csrc/relay/relay.cpp) built with AddressSanitizer + UBSan (host code, g++)
runs the relay contract tests and a burst of concurrent streams with client disconnects: any
memory error or undefined behaviour aborts the relay process and fails the test."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "llmd_amd", "csrc", "relay", "relay.cpp")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def test_relay_under_asan_ubsan(tmp_path):
    exe = tmp_path / "llmd-relay-asan"
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", SRC, "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, LLMD_RELAY_BIN=str(exe), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_router_relay.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout
