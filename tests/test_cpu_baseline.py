"""The optimised CPU baseline (oracle/ewal_cpu_fast.c, bench.py's
cpu_baseline "optimised" leg) returns the faithful restatement's results on
every input it accepts -- otherwise its timings would not be of the same
work.  CPU only."""
import ctypes as C
import random

import numpy as np

from oracle import oracle as O
from test_gpu_parity import build_wal


def _both(buf, ri):
    o = O.readall_digest(buf, ri)
    for th in (1, 3):
        f = O.fast_readall(buf, ri, th)
        if f is None:
            return o, None
        assert f == o, (th, f, o)
    return o, f


def test_fast_readall_random_wals():
    rng = random.Random(11)
    hit = 0
    for i in range(60):
        w = build_wal(rng, rng.randrange(0, 200), rng.choice([10, 300, 5000, 70000]), cuts=rng.randrange(0, 3))
        ri = rng.choice([0, 0, 1, 5, 10 ** 6])
        _, f = _both(w, ri)
        hit += f is not None
        bad = bytearray(w)
        if len(bad) > 40:
            bad[rng.randrange(30, len(bad))] ^= 1 << rng.randrange(8)
            _both(bytes(bad), ri)
    assert hit >= 40


def test_fast_readall_error_classes():
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"m1")
    e.save_entry(0, 1, 0, b"x")
    e.encode(1, b"m2")
    o, f = _both(e.getvalue(), 0)
    assert o["status"] == O.ERR_METADATA_CONFLICT and f is not None
    a = O.WalEncoder(0)
    a.save_crc(0)
    a.encode(1, b"m")
    a.save_entry(0, 1, 0, b"abc")
    b = O.WalEncoder(a.crc ^ 1)
    b.save_crc(0)
    o, f = _both(a.getvalue() + b.getvalue(), 0)
    assert o["status"] == O.ERR_WAL_CRC and f is not None
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(9, b"payload")
    o, f = _both(e.getvalue(), 0)
    assert o["status"] == O.ERR_UNEXPECTED_TYPE and f is not None and f["detail"] == 9
    # metadata != nil && !DeepEqual: a nil first metadata disables the check,
    # a nil one after a non-nil one conflicts
    e = O.WalEncoder(0)
    e.encode(1, None)
    e.encode(1, b"x")
    o, f = _both(e.getvalue(), 0)
    assert o["status"] == O.OK and f is not None
    e.encode(1, None)
    o, f = _both(e.getvalue(), 0)
    assert o["status"] == O.ERR_METADATA_CONFLICT and f is not None
    # torn tail / index gap: outside the fast path, never a different answer
    w = build_wal(random.Random(3), 20, 100)
    assert O.fast_readall(w[:-3], 0, 2) is None
    e = O.WalEncoder(0)
    e.save_entry(0, 1, 5, b"a")
    assert O.fast_readall(e.getvalue(), 0, 1) is None


def test_fast_crc32c():
    rng = random.Random(5)
    for n in (0, 1, 7, 8, 12287, 12288, 12289, 40000, 200001):
        d = rng.randbytes(n)
        c = rng.getrandbits(32)
        assert O.fast_crc32c(c, d) == O.crc32_update(c, d)


def test_fast_batches():
    rng = random.Random(7)
    shards = [build_wal(rng, rng.randrange(1, 60), 3000) for _ in range(9)]
    shards[4] = bytearray(shards[4])
    shards[4][-2] ^= 0x10
    shards[4] = bytes(shards[4])
    blob = b"".join(shards)
    offs = [sum(len(s) for s in shards[:i]) for i in range(len(shards))]
    raw = C.create_string_buffer(blob, len(blob))
    st, fr = O.fast_readall_batch(C.addressof(raw), offs, [len(s) for s in shards], 0, 4)
    st2, fr2 = O.fast_readall_batch(C.addressof(raw), offs, [len(s) for s in shards], 0, 4, faithful=True)
    for s, x, y, x2, y2 in zip(shards, st, fr, st2, fr2):
        o = O.readall_digest(s, 0)
        assert x == x2 == o["status"] and y == y2 == (o["n_records"] if o["status"] == O.OK else o["fail_record"])
    files = []
    for i in range(7):
        body = O.snapshot_marshal(rng.randbytes(rng.randrange(0, 50000)), [1, 2], i, 1)
        f = bytearray(O.snappb_marshal(O.crc32_update(0, body), body))
        if i == 3:
            f[-5] ^= 0x20
        files.append(bytes(f))
    blob = b"".join(files)
    offs = [sum(len(s) for s in files[:i]) for i in range(len(files))]
    raw = C.create_string_buffer(blob, len(blob))
    st, cc = O.fast_snap_verify_batch(C.addressof(raw), offs, [len(f) for f in files], 3)
    for f, x, c in zip(files, st, cc):
        o = O.loadsnap(f)
        assert x == o["status"] and c == o["computed_crc"]


def test_fast_commit_batch():
    rng = np.random.default_rng(6)
    G = 4000
    nv = rng.choice([1, 3, 5, 7, 9], size=G).astype(np.uint8)
    match = rng.integers(0, 40, size=(9, G), dtype=np.uint64).reshape(-1)
    term = rng.integers(1, 4, size=G, dtype=np.uint64)
    c0 = rng.integers(0, 20, size=G, dtype=np.uint64)
    off = rng.integers(0, 5, size=G, dtype=np.uint64)
    ptr = np.arange(G + 1, dtype=np.uint64) * np.uint64(16)
    lt = np.sort(rng.integers(1, 4, size=(G, 16), dtype=np.uint64), axis=1).reshape(-1)
    ca, cb = c0.copy(), c0.copy()
    cha, chb, sta, stb = (np.zeros(G, np.uint8) for _ in range(4))
    O.maybe_commit_batch(G, match, nv, term, ca, off, ptr, lt, cha, sta)
    O.fast_maybe_commit_batch(G, match, nv, term, cb, off, ptr, lt, chb, stb, 4)
    assert (ca == cb).all() and (cha == chb).all() and (sta == stb).all()
