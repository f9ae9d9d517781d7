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


def _join_line(rows, blobs, rig):
    """The san_join output line of one case, from libewal.so's own join."""
    import ctypes as C
    from etcd_amd import _lib as L
    n = len(rows)
    arr = (L.RangeRow * max(n, 1))(*rows)
    md = b"".join(blobs)
    out = L.SplitResult()
    rc = L.lib.ewal_split_verdict(arr, n, rig & (2 ** 64 - 1), md, len(md), C.byref(out))
    if rc:
        return "rc %d" % rc
    s = "%d %d %d %d %d %d %d %d %d %d %d |" % (out.status, out.fail_record, out.n_records, out.resplit, out.last_crc,
                                               out.enti, out.md_range, out.md_blob_off, out.md_len, out.state_range,
                                               out.n_ents)
    if out.status == L.OK and out.resplit < 0:
        base, cnt = (C.c_int64 * max(n, 1))(), (C.c_int64 * max(n, 1))()
        ln = L.lib.ewal_split_ents_layout(arr, n, rig & (2 ** 64 - 1), base, cnt)
        s += " %d" % ln + "".join(" %d:%d" % (base[k], cnt[k]) for k in range(n))
    return s


def _join_cases():
    """By-file splits of the split suites' WALs (clean, corrupt, torn, seam,
    metadata, index rules, mutated, the entry-less last file with an unknown-
    field HardState) over 2-4 ranges, each resplit followed to its final
    verdict: [(rows, md blobs, w.ri)]."""
    import random
    import struct
    from oracle import oracle as O
    from etcd_amd import shard
    from test_split_wal import _cases, _mutated_cases, oracle_range_info
    from test_split_join import _state_only_last_file

    def rows_of(parts):
        rr = [shard.range_row(tuple(O.readall(b, ri)[k] for k in ("status", "fail_record", "n_records", "last_crc")),
                              oracle_range_info(b, ri), ri) for b, ri in parts]
        return [r for r, _ in rr], [m for _, m in rr]

    out = []
    for world in (2, 3, 4):
        rng = random.Random(90 + world)
        cases = _cases(rng, world) + _mutated_cases(rng, world, n=6)
        files = _state_only_last_file(rng, nfiles=world + 1)
        per = [(files[0][0], 1)] + [(b"".join(b for b, _ in files[1:world]), max(1, files[1][1]))]
        per += [(files[-1][0], max(1, files[-1][1]))] + [(b"", 0)] * (world - 2)
        cases.append((b"".join(b for b, _ in files), 1, per[:world + 1] if world > 2 else per[:3]))
        for _, rig, parts in cases:
            for _ in range(len(parts) + 1):   # follow the join's resplits
                rows, blobs = rows_of(parts)
                out.append((rows, blobs, rig))
                v = shard.join_rows(rows, blobs, rig)
                if v[3] < 0:
                    break
                k = v[3]
                parts = parts[:k] + [(b"".join(b for b, _ in parts[k:]), parts[k][1])] + [(b"", 0)] * (len(parts) - k - 1)
    del struct
    return out


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_split_join_under_asan_ubsan(tmp_path):
    """the host-only join of ONE WAL read as several ranges
    (ewal_split_verdict, ewal_split_ents_layout: md blob offsets, ents
    truncation across ranges, resplits) built with ASan + UBSan and driven over
    the split suites' rows (every case's resplits followed); its output must
    equal libewal.so's own join on the same rows."""
    import struct
    exe = str(tmp_path / "san_join")
    _run(["g++", "-std=c++17", *SAN, "-I", os.path.join(ROOT, "include"), "-o", exe,
          os.path.join(HERE, "sanitize", "san_join.cpp"), os.path.join(ROOT, "etcd_amd", "csrc", "ewal_join.cpp"),
          os.path.join(ROOT, "etcd_amd", "csrc", "ewal_host.cpp"), os.path.join(HERE, "sanitize", "join_gpu_stubs.cpp"),
          "-lpthread"])
    cases = _join_cases()
    assert len(cases) > 60
    want = []
    with open(tmp_path / "rows.bin", "wb") as f:
        for rows, blobs, rig in cases:
            md = b"".join(blobs)
            f.write(struct.pack("<QQQ", len(rows), rig & (2 ** 64 - 1), len(md)) + md)
            for r in rows:
                f.write(bytes(r))
            want.append(_join_line(rows, blobs, rig))
    p = subprocess.run([exe, str(tmp_path / "rows.bin")], capture_output=True, text=True, env=ENV, timeout=300)
    assert p.returncode == 0, p.stderr[-6000:]
    assert "san_join ok (%d cases)" % len(cases) in p.stderr
    got = [x.rstrip() for x in p.stdout.splitlines()]
    assert got == [x.rstrip() for x in want]
    assert any(not x.startswith("rc") and x.split()[3] != "-1" for x in want)   # resplits among the cases
