"""The device-free host C++ of libfdlp_hip.so (fdlp_host.cpp: RNG replicas, noise energies, the WAV decoder
on well-formed, truncated and corrupted buffers, the atomic ark writer, the Kaldi matrix reader/writer)
built with AddressSanitizer + UndefinedBehaviorSanitizer and run on the CPU (sanitizers on
the host code)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    src = [os.path.join(ROOT, "tests", "sanitize", "host_sanitize.cpp"),
           os.path.join(ROOT, "speech_recognition_tools_amd", "csrc", "fdlp_host.cpp")]
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-o", exe] + src,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    # verify_asan_link_order=0: the environment may preload other libraries ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "host sanitizer checks passed" in r.stdout
