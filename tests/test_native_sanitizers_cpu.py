"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer.

GPU sanitizers (xnack+ ASan) are not available on the MI355X pool, so the sanitized target is the
host C++ runtime: the text pipeline core (``csrc/runtime/text_core.h``, the same header the
extension compiles) driven by ``tests/native/text_core_check.cpp`` over its edge cases.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "performance-comparison-of-tensorflow-pytorch-and-their-distributed-counterparts_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_text_core_under_asan_ubsan(tmp_path):
    exe = tmp_path / "text_core_check"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{CSRC}", os.path.join(ROOT, "tests", "native", "text_core_check.cpp"),
           "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "text_core_check: ok" in r.stdout
