"""Host C++ runtime under AddressSanitizer + UndefinedBehaviorSanitizer.

csrc/host/csv.cpp (CSV index / fields / type inference / typed parse / dictionary encoding, word
count) is linked with csrc/host_tests/csv_sanitize_main.cpp into a standalone sanitized executable
and run over the reference's health.csv fixture plus seeded fuzz buffers.  No preload or Python
interposition is involved: the executable carries its own sanitizer runtime."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_runtime_asan_ubsan(tmp_path):
    exe = tmp_path / "csv_sanitize"
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "csrc", "host"),
           os.path.join(ROOT, "csrc", "host", "csv.cpp"), os.path.join(ROOT, "csrc", "host_tests", "csv_sanitize_main.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([str(exe), os.path.join(ROOT, "tests", "data", "health.csv"), "--fuzz", "300"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "SANITIZE_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
