"""ASan + UBSan runs of the host code (CPU only): the oracle and optimised
CPU baseline (oracle/*.c) and the engine's host C++ (etcd_amd/csrc/
ewal_host.cpp) are compiled with -fsanitize=address,undefined and driven over
random and corrupted inputs (tests/sanitize/).  The reference runs its tests
under `go test --race`; GPU sanitizers are not available on
the MI355X pool, so the device code is covered by the parity suites."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def _run(cmd, **kw):
    p = subprocess.run(cmd, capture_output=True, text=True, **kw)
    assert p.returncode == 0, (cmd, p.stdout[-3000:], p.stderr[-6000:])
    return p.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_oracle")
    _run(["gcc", "-std=c11", *SAN, "-o", exe, os.path.join(HERE, "sanitize", "san_oracle.c"),
          os.path.join(ROOT, "oracle", "ewal_oracle.c"), os.path.join(ROOT, "oracle", "ewal_cpu_fast.c"), "-lpthread"])
    out = _run([exe], env=ENV, timeout=300)
    assert "san_oracle ok" in out


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_cpp_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_host")
    _run(["g++", "-std=c++17", *SAN, "-I", os.path.join(ROOT, "include"), "-o", exe,
          os.path.join(HERE, "sanitize", "san_host.cpp"), os.path.join(ROOT, "etcd_amd", "csrc", "ewal_host.cpp"),
          os.path.join(ROOT, "etcd_amd", "csrc", "ewal_synth.cpp"), "-lpthread"])
    out = _run([exe, str(tmp_path / "wal")], env=ENV, timeout=300)
    assert "san_host ok (0 failures)" in out
