"""Sanitizer builds of the native host runtime: the C++ self-test
(csrc/runtime/tests/selftest.cpp) is compiled together with the runtime sources under
AddressSanitizer + UndefinedBehaviorSanitizer, and under ThreadSanitizer (races between the ring's
producer and consumer threads), then executed.  Host code only -- GPU sanitizers are not used."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "csrc", "runtime", f) for f in ("sumtree.cpp", "ipc.cpp")]
TEST = os.path.join(ROOT, "csrc", "runtime", "tests", "selftest.cpp")


def _build_and_run(tmp_path, flags, env_extra):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "selftest")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, TEST, *SRCS,
           "-o", exe, "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest ok" in r.stdout


def test_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1:verify_asan_link_order=0"})


def test_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
