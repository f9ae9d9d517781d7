"""The cgo shim's call sequence (INTEGRATION.md readAllGPU), as a C program
linked against libewal.so (tests/shim/readall_shim.c): OpenAtIndex over a
WAL directory the engine's writer produced, ReadAll, the Go sentinel switch
and the zero-copy materialisation of ents -- against the oracle's ReadAll
over the same files (wal/wal.go:108-216; TestRecover / TestRecoverAfterCut /
TestOpenAtUncommittedIndex shapes, wal/wal_test.go:152-351)."""
import json
import os
import random
import struct
import subprocess

import pytest

from oracle import oracle as O
from etcd_amd import wal as W

HERE = os.path.dirname(os.path.abspath(__file__))
SHIM = os.path.join(HERE, "shim", "readall_shim")


def run_shim(d, index):
    assert os.path.exists(SHIM), "build() compiles tests/shim/readall_shim"
    p = subprocess.run([SHIM, str(d), str(index)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def expected(d, index):
    """OpenAtIndex's file selection (wal/wal.go:108-159, util.go:20-49)
    restated here, then the oracle's ReadAll with w.ri = index."""
    names = sorted(n for n in os.listdir(d) if n.endswith(".wal"))
    parsed = [(int(n[:16], 16), int(n[17:33], 16)) for n in names]
    ni = next((i for i in range(len(parsed) - 1, -1, -1) if index >= parsed[i][1]), -1)
    if ni < 0:
        return None
    seqs = [s for s, _ in parsed[ni:]]
    if any(seqs[k] != seqs[k - 1] + 1 for k in range(1, len(seqs)) if seqs[k - 1] != 0):
        return None
    buf = b"".join(open(os.path.join(d, n), "rb").read() for n in names[ni:])
    return O.readall_digest(buf, index)


def check(d, index):
    g = run_shim(d, index)
    o = expected(d, index)
    if o is None:
        assert g["sentinel"] == "wal.ErrFileNotFound", g
        return g
    assert g["rc"] == o["status"], (g, o["status"])        # the status numbering is the oracle's
    if o["status"] == O.OK:
        assert (g["n_records"], g["n_ents"], g["enti"], g["last_crc"]) == \
            (o["n_records"], o["n_ents"], o["enti"], o["last_crc"])
        assert g["ents_digest"] == o["ents_digest"]
        assert tuple(g["state"]) == o["state"]
        assert g["metadata_len"] == (len(o["metadata"]) if o["metadata"] is not None else -1)
    elif o["status"] != O.ERR_INDEX_NOT_FOUND:
        assert g["fail_record"] == o["fail_record"]
    return g


@pytest.mark.gpu
def test_shim_recover_after_cut(tmp_path):
    d = tmp_path / "wal"
    rng = random.Random(5)
    w = W.Create(str(d), b"metadata")
    idx = 0
    for f in range(10):
        cnt = rng.randrange(1, 400)
        w.Save(W.HardState(1, 1, idx), [W.Entry(0, 1, idx + k, rng.randbytes(rng.randrange(0, 3000)))
                                         for k in range(cnt)])
        idx += cnt
        w.Cut()
    w.Close()
    names = sorted(os.listdir(d))
    assert len(names) == 11
    for index in (0, 1, 5, 250, 10 ** 6):
        check(d, index)
    # TestRecoverAfterCut: a file in the middle removed
    os.remove(d / names[4])
    first4 = int(names[4][17:33], 16)
    g = check(d, 0)
    assert g["sentinel"] == "wal.ErrFileNotFound"
    g = check(d, first4)
    assert g["sentinel"] == "wal.ErrFileNotFound"
    nxt = int(names[5][17:33], 16)
    g = check(d, nxt)
    assert g["sentinel"] == "nil" and g["n_ents"] > 0


@pytest.mark.gpu
def test_shim_large_and_corrupt(tmp_path):
    d = tmp_path / "wal"
    os.makedirs(d)
    buf, n = W.synth_wal(64 << 20, 64, 65536, seed=9)
    (d / W.walName(0, 0)).write_bytes(bytes(buf))
    g = check(d, 1)
    assert g["sentinel"] == "nil" and g["n_ents"] > 1000 and g["ms"]["total"] > 0
    bad = bytearray(buf)
    bad[len(bad) // 2] ^= 0x40
    (d / W.walName(0, 0)).write_bytes(bytes(bad))
    g = check(d, 1)
    assert g["sentinel"] != "nil"


def unrec_digest(o):
    """The shim's XXX_unrecognized digest over the oracle's ReadAll result."""
    h = 0
    items = [(i, e["unrec"]) for i, e in enumerate(o["ents"]) if e["unrec"] is not None]
    if o["state"]["unrec"] is not None:
        items.append(((1 << 64) - 1, o["state"]["unrec"]))
    for who, b in items:
        h = O.crc32_update(h, struct.pack("<QQ", who, len(b)))
        h = O.crc32_update(h, b)
    return h, len(items)


@pytest.mark.gpu
def test_shim_unknown_fields(tmp_path):
    """Entries and the HardState carrying unknown fields: the shim returns their
    XXX_unrecognized (raft.pb.go:273,699) byte-exact, as reflect.DeepEqual in
    wal_test.go:188 would see them."""
    d = tmp_path / "wal"
    os.makedirs(d)
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"metadata")
    for i in range(40):
        tail = bytes([0x38, i]) if i % 3 == 0 else (bytes([0x45, 1, 2, 3, i]) if i % 7 == 0 else b"")
        e.encode(2, O.entry_marshal(0, 1, i, bytes([i]) * (i * 13 % 300)) + tail)
    e.encode(3, O.hardstate_marshal(1, 2, 30) + bytes([0x20, 0x07]))
    buf = e.getvalue()
    (d / W.walName(0, 0)).write_bytes(buf)
    g = check(d, 0)
    o = O.readall(buf, 0)
    assert o["status"] == O.OK and g["sentinel"] == "nil"
    assert (g["unrec_digest"], g["n_unrec"]) == unrec_digest(o)
    assert g["n_unrec"] > 10


@pytest.mark.gpu
def test_shim_damaged_directories(tmp_path):
    # a WAL directory the engine's writer produced, one file damaged by
    # test_gpu_fuzz's mutations: the shim's sentinel, failing frame and
    # materialised ents must be the oracle's ReadAll over the selected files
    from test_gpu_fuzz import _mutate
    rng = random.Random(23)
    for case in range(8):
        d = tmp_path / ("wal%d" % case)
        w = W.Create(str(d), b"metadata")
        idx = 0
        for f in range(rng.randrange(2, 5)):
            cnt = rng.randrange(5, 120)
            w.Save(W.HardState(1, 1, idx), [W.Entry(0, 1, idx + k, rng.randbytes(rng.randrange(0, 1500)))
                                             for k in range(cnt)])
            idx += cnt
            w.Cut()
        w.Close()
        names = sorted(os.listdir(d))
        victim = d / names[rng.randrange(len(names))]
        victim.write_bytes(_mutate(rng, victim.read_bytes()))
        for index in (0, rng.randrange(1, idx + 1)):
            check(d, index)


def run_shim_mode(d, index, mode):
    p = subprocess.run([SHIM, str(d), str(index), mode], capture_output=True, text=True, timeout=180)
    return p


@pytest.mark.gpu
def test_shim_overlap_ctx_exits_cleanly(tmp_path):
    """EWAL_OPT_OVERLAP through the C ABI (a WAL large enough for the frame
    pass's 1 MiB tiles, >= 6 GiB on 256 CUs: the chunked, CU-masked pipeline
    runs, so frames_ms is 0): the results are the oracle's, and the process
    exits 0 both after ewal_ctx_destroy and with the ctx left alive (the
    library's atexit teardown of its masked streams; round 5 saw a SIGSEGV in
    __cxa_finalize for a live overlap ctx).  The WAL file lives in tmpfs."""
    import shutil
    import tempfile
    base = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    d = tempfile.mkdtemp(prefix="ewal_ov_", dir=base)
    try:
        _overlap_modes(d)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _overlap_modes(d):
    buf, n = W.synth_wal((6 << 30) + (64 << 20), 64, 65536, seed=21)
    with open(os.path.join(d, W.walName(0, 0)), "wb") as f:
        f.write(memoryview(buf))
    o = O.readall_digest(bytes(buf), 1)
    del buf
    for mode in ("overlap", "overlap-live"):
        p = run_shim_mode(d, 1, mode)
        assert p.returncode == 0, (mode, p.returncode, p.stderr[-2000:])
        g = json.loads(p.stdout.strip().splitlines()[-1])
        assert g["rc"] == o["status"] == O.OK, (mode, g)
        assert (g["n_records"], g["n_ents"], g["enti"], g["last_crc"], g["ents_digest"]) == \
            (o["n_records"], o["n_ents"], o["enti"], o["last_crc"], o["ents_digest"]), mode
        assert g["frames_ms"] == 0.0, (mode, g)   # the overlapped pipeline ran (no single frame-pass launch)
