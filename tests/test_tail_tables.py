"""Host check of the frame pass's shift tables (etcd_amd/csrc/crc_math.h
EW_TAIL_TABS): every table against direct CRC-32C register arithmetic, and
the identities the GPU code builds on them -- the masked-block prefix tail
(wal_kernels.hip prefix_near_tail) and the checks' three-round S_dlen
(frame_kernels.hip).  CPU only: the GPU parity suites check the kernels."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_tail_tables_and_identities(tmp_path):
    exe = str(tmp_path / "tail_tables")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "etcd_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tests", "host", "tail_tables.cpp")], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
