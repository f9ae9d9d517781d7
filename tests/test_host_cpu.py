"""CPU-side checks of the product (no GPU): the C-ABI library loads and exports
every symbol include/ewal.h declares; the host write path, file selection and
synthetic generator agree byte-for-byte with the oracle; compute entry points
fail loudly (EWAL_E_NODEVICE) instead of falling back to the CPU."""
import ctypes as C
import os
import random

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W


def test_library_exports_every_header_symbol():
    syms = L.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L.lib, s)]
    assert not missing, missing


def test_status_codes_match_oracle():
    for name in ("OK", "EOF", "ERR_UNEXPECTED_EOF", "ERR_RECORD_CRC", "ERR_WAL_CRC", "ERR_METADATA_CONFLICT",
                 "ERR_INDEX_NOT_FOUND", "ERR_WRONG_TYPE", "ERR_UNEXPECTED_TYPE", "ERR_FILE_NOT_FOUND", "ERR_SNAP_CRC",
                 "ERR_NO_SNAPSHOT", "PANIC_NEG_LENGTH", "PANIC_BOUNDS", "PANIC_ENTRY", "PANIC_STATE",
                 "PANIC_INDEX_GAP", "NONTERMINATING"):
        assert getattr(L, name) == getattr(O, name), name


def test_host_crc_matches_oracle():
    rng = random.Random(7)
    for n in (0, 1, 7, 8, 63, 4096, 3 * 4096 + 5, 100000):
        d = bytes(rng.getrandbits(8) for _ in range(n))
        seed = rng.getrandbits(32)
        for poly in (L.CASTAGNOLI, L.IEEE, L.KOOPMAN):
            assert L.lib.ewal_crc32_update_host(seed, poly, d, n) == O.crc32_update(seed, d, poly)


def test_crc_combine():
    rng = random.Random(3)
    for _ in range(50):
        a = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        b = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        seed = rng.getrandbits(32)
        ca = O.crc32_update(seed, a)
        cb = O.crc32_update(0, b)
        assert L.lib.ewal_crc32_combine(L.CASTAGNOLI, ca, cb, len(b)) == O.crc32_update(seed, a + b)


def test_encoder_matches_oracle_bytes():
    rng = random.Random(11)
    e = W.Encoder(0)
    o = O.WalEncoder(0)
    e.encode(4, None)
    o.encode(4, None)
    e.encode(1, b"metadata")
    o.encode(1, b"metadata")
    for i in range(200):
        d = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 2000))) if rng.random() < 0.9 else None
        e.save_entry(rng.choice([0, 1]), rng.randrange(1 << 40), i, d)
    # rebuild the oracle stream deterministically with the same calls
    rng = random.Random(11)
    o = O.WalEncoder(0)
    o.encode(4, None)
    o.encode(1, b"metadata")
    for i in range(200):
        d = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 2000))) if rng.random() < 0.9 else None
        o.save_entry(rng.choice([0, 1]), rng.randrange(1 << 40), i, d)
    e.save_state(3, 2, 1)
    o.save_state(3, 2, 1)
    e.save_state(0, 0, 0)   # IsEmptyHardState: not written
    o.save_state(0, 0, 0)
    assert e.getvalue() == o.getvalue()
    assert e.crc == o.crc


def test_synth_wal_is_valid_and_corruption_lands():
    buf, n = W.synth_wal(1 << 20, 64, 4096, seed=5)
    # entries carry Index 1..N, so the replay starts at ri = 1 (ri = 0 would hit
    # the reference's ents[:1] slice panic on an empty slice, wal/wal.go:173)
    assert O.readall(bytes(buf), 0)["status"] == O.PANIC_INDEX_GAP
    r = O.readall(bytes(buf), 1)
    assert r["status"] == O.OK and r["n_records"] == n
    assert [e["index"] for e in r["ents"]] == list(range(1, n - 2))
    assert r["metadata"] == b"\x08\x01" and r["state"] == dict(term=1, vote=1, commit=0, unrec=None)
    bad, n2 = W.synth_wal(1 << 20, 64, 4096, seed=5, corrupt_record=17)
    r2 = O.readall(bytes(bad), 1)
    assert n2 == n and r2["status"] == O.ERR_RECORD_CRC and r2["fail_record"] == 17


def test_writer_dir_matches_oracle(tmp_path):
    d = str(tmp_path / "wal")
    w = W.Create(d, b"metadata")
    w.SaveEntry(W.Entry(0, 0, 0, None))
    w.Cut()
    for i in range(1, 6):
        w.SaveEntry(W.Entry(0, 1, i, bytes([i])))
        w.Cut()
    w.SaveState(W.HardState(1, 1, 5))
    w.Close()
    names = sorted(os.listdir(d))
    assert names[:3] == ["0000000000000000-0000000000000000.wal", "0000000000000001-0000000000000001.wal",
                         "0000000000000002-0000000000000002.wal"]
    whole = b"".join(open(os.path.join(d, x), "rb").read() for x in names)
    r = O.readall(whole, 0)
    assert r["status"] == O.OK and [e["index"] for e in r["ents"]] == list(range(6))
    assert r["state"] == dict(term=1, vote=1, commit=5, unrec=None)
    with pytest.raises(FileExistsError):
        W.Create(d, None)


def test_open_at_index_file_selection(tmp_path):
    # TestOpenAtIndex (wal/wal_test.go:60-112) + TestRecoverAfterCut's missing file
    d = str(tmp_path / "w")
    os.makedirs(d)
    open(os.path.join(d, "0000000000000000-0000000000000000.wal"), "wb").close()
    assert W.OpenAtIndex(d, 0).seq == 0
    open(os.path.join(d, "0000000000000002-000000000000000a.wal"), "wb").close()
    # isValidSeq skips the check while lastSeq == 0 (wal/util.go:36-49), so
    # seq 0 -> 2 is accepted and the WAL appends to the seq-2 file
    assert W.OpenAtIndex(d, 5).seq == 2
    assert W.OpenAtIndex(d, 10).seq == 2
    open(os.path.join(d, "0000000000000004-0000000000000014.wal"), "wb").close()
    with pytest.raises(L.EwalError) as ei:
        W.OpenAtIndex(d, 10)          # seq 2 -> 4 is a gap
    assert ei.value.status == L.ERR_FILE_NOT_FOUND
    e = str(tmp_path / "empty")
    os.makedirs(e)
    with pytest.raises(L.EwalError) as ei:
        W.OpenAtIndex(e, 0)
    assert ei.value.status == L.ERR_FILE_NOT_FOUND


def test_compute_fails_loudly_without_gpu():
    if L.lib.ewal_device_count() > 0:
        pytest.skip("a GPU is present")
    p = C.c_void_p()
    assert L.lib.ewal_ctx_create(0, C.byref(p)) == L.E_NODEVICE


def test_snapshot_writer_matches_oracle():
    """etcd_amd.snap (Snapshotter.save, snap/snapshotter.go:46-60) byte-identical to the oracle's marshal."""
    from etcd_amd import snap as S
    rng = random.Random(3)
    for n in (0, 1, 127, 128, 5000):
        data = bytes(rng.getrandbits(8) for _ in range(n))
        nodes = [rng.randrange(1, 1 << 40) for _ in range(rng.randrange(0, 4))]
        index, term = rng.randrange(1 << 30), rng.randrange(1 << 20)
        body = S.snapshot_marshal(data, nodes, index, term, (7,))
        assert body == O.snapshot_marshal(data, nodes, index, term, (7,))
        f = S.snap_file(body)
        assert f == O.snappb_marshal(O.crc32_update(0, body), body)
        assert O.loadsnap(f)["status"] == O.OK


def test_commit_batch_oracle_matches_per_group():
    """The CPU baseline's batched maybeCommit equals the per-group restatement (raft/raft.go:248-258)."""
    import numpy as np
    rng = np.random.default_rng(1)
    G = 2000
    nv = rng.choice(np.array([0, 1, 2, 3, 5, 7, 16], dtype=np.uint8), size=G)
    match = rng.integers(0, 30, size=(16, G), dtype=np.uint64)
    term = rng.integers(1, 4, size=G, dtype=np.uint64)
    c0 = rng.integers(0, 20, size=G, dtype=np.uint64)
    off = rng.integers(0, 10, size=G, dtype=np.uint64)
    lens = rng.integers(0, 20, size=G)
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    lt = np.sort(rng.integers(1, 4, size=int(ptr[-1]), dtype=np.uint64))
    c = c0.copy()
    ch, st = np.zeros(G, np.uint8), np.zeros(G, np.uint8)
    O.maybe_commit_batch(G, match.reshape(-1), nv, term, c, off, ptr, lt, ch, st)
    for g in range(G):
        rc, want = O.maybe_commit([int(match[v, g]) for v in range(nv[g])], int(term[g]), int(c0[g]),
                                  [int(x) for x in lt[ptr[g]:ptr[g + 1]]], int(off[g]))
        if rc < 0:
            assert st[g] == -rc
        else:
            assert (st[g], ch[g], c[g]) == (0, rc, want), g


def test_synth_shards_layout():
    blob, lens, nrec = W.synth_shards([5, 6, 7], 1 << 16, 128, 4096, corrupt={1: 3})
    assert len(blob) == sum(lens)
    pos = 0
    for i, (n, k) in enumerate(zip(lens, nrec)):
        shard = bytes(blob[pos:pos + n])
        one, kk = W.synth_wal(1 << 16, 128, 4096, seed=5 + i, corrupt_record=3 if i == 1 else -1)
        assert shard == bytes(one) and k == kk
        o = O.readall(shard, 1)
        assert o["status"] == (O.ERR_RECORD_CRC if i == 1 else O.OK)
        pos += n


def test_message_writer_matches_oracle():
    """etcd_amd.raftmsg marshal (raft.pb.go:921-943, 1010-1068) byte-identical to the oracle's."""
    from etcd_amd import raftmsg as M
    from etcd_amd import snap as S
    rng = random.Random(8)
    for _ in range(50):
        ents = [(rng.choice([0, 1]), rng.randrange(1 << 40), rng.randrange(1 << 40),
                 bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3, 200])))) for _ in range(rng.randrange(4))]
        mine = [M.entry_marshal(*e) for e in ents]
        assert mine == [O.entry_marshal(*e) for e in ents]
        snap = S.snapshot_marshal(b"s" * rng.randrange(5), (1, 2), 3, 4)
        args = (rng.randrange(16), rng.randrange(1 << 63), rng.randrange(1 << 20), rng.randrange(1 << 30),
                rng.randrange(1 << 30), rng.randrange(1 << 40))
        rej = rng.random() < 0.5
        assert M.message_marshal(*args, mine, 77, snap, rej) == O.message_marshal(*args, mine, 77, snap, rej)


def test_shim_harness_links_and_fails_loudly_without_gpu():
    """tests/shim/readall_shim (the cgo shim's call sequence in C) links
    against libewal.so; without a GPU it reports EWAL_E_NODEVICE at context
    creation -- no CPU fallback."""
    import json
    import subprocess
    shim = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shim", "readall_shim")
    if not os.path.exists(shim):
        pytest.skip("build() not run")
    p = subprocess.run([shim, "/nonexistent", "0"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0
    out = json.loads(p.stdout.strip().splitlines()[-1])
    if L.lib.ewal_device_count() == 0:
        assert out["ok"] is False and out["rc"] == L.E_NODEVICE


def test_commit_records_pack():
    """raftcommit.pack_groups: the 192-B ecommit_group rows (include/ewal.h)
    hold the voters' Match, committed, Term, the log bounds and the terms of
    the log's last 13 entries -- checked field by field on a small batch."""
    import numpy as np
    from etcd_amd import raftcommit as RC
    rng = np.random.default_rng(3)
    G = 50
    nv = rng.integers(1, 8, size=G).astype(np.uint8)
    match = rng.integers(0, 1 << 40, size=(7, G), dtype=np.uint64)
    c0 = rng.integers(0, 1 << 30, size=G, dtype=np.uint64)
    term = rng.integers(1, 9, size=G, dtype=np.uint64)
    off = rng.integers(0, 1 << 30, size=G, dtype=np.uint64)
    lens = rng.integers(0, 20, size=G).astype(np.uint64)
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    lt = rng.integers(1, 1 << 20, size=int(lens.sum()), dtype=np.uint64)
    rec = RC.pack_groups(match, nv, c0, term, off, ptr, lt)
    assert rec.shape == (G, 24) and rec.dtype == np.uint64
    for g in range(G):
        assert list(rec[g, :7]) == list(match[:, g])
        assert (rec[g, 7], rec[g, 8], rec[g, 9]) == (c0[g], term[g], off[g])
        assert int(rec[g, 10]) == int(lens[g]) | (int(nv[g]) << 32)
        for k in range(13):
            want = lt[int(ptr[g + 1]) - 1 - k] if k < lens[g] else 0
            assert rec[g, 11 + k] == want
