"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY
§5.2): the C++ block manager / KV index / GBDT / FS store are compiled into an
instrumented executable that embeds CPython and runs the randomised stress
driver tests/native/rt_stress.py. The same driver also runs against the
normal extension."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "native"))


def test_stress_plain():
    import rt_stress

    from llmd_amd import _rt_loader

    res = rt_stress.run_all(_rt_loader.rt())
    assert res["fs"] == 40 and res["gbdt_mae"] < 0.5


def test_runtime_asan_ubsan():
    from llmd_amd.build import build_sanitized_runtime

    exe = build_sanitized_runtime()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), os.path.join(ROOT, "tests", "native", "rt_stress.py")], env=env,
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert "rt_sanitize ok" in out
