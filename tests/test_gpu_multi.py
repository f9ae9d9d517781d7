"""ONE WAL split over several contexts in one process (ewal_multi_readall /
ewal_multi_readall_device): one host thread per ctx -- here 2 and 3 ctxs on device 0 --
each reading its range (whole files, or a range opening at a frame-start
candidate inside a file with frame 0's check deferred), and ReadAll's
cross-range rules joined in the C ABI (ewal_split_verdict, the join
etcd_amd/shard.py also calls after its torch.distributed exchange).  The
joined verdict must be the oracle's ReadAll over the whole WAL, on clean and
on damaged WALs (test_gpu_fuzz's mutations), and on the two cases ADVICE r03
found in the Python join: a range whose frame 0 fails its Entry decode (that
comes after decoder.decode's CRC check, so the deferred CRC check wins) and a
file ending in a bare length prefix (io.EOF for the range alone).  Since
round 5 the join returns ReadAll's whole result -- metadata, HardState and
the ents stitched across the ranges (ewal_split_ents_layout) -- and every
field is compared with the oracle's; a 1 GiB configs[1]-shaped WAL split
in HBM (no copy) must give the single-ctx ReadAll exactly."""
import random
import struct

import pytest

from oracle import oracle as O
from etcd_amd import shard
from etcd_amd import wal as W
from test_gpu_fuzz import _mutate
from test_split_wal import build_files
from test_split_within_file import _wal

pytestmark = pytest.mark.gpu


def _want(buf, ri):
    o = O.readall(buf, ri)
    return o["status"], (o["fail_record"] if o["status"] not in (O.OK, O.ERR_INDEX_NOT_FOUND) else -1), o["n_records"]


@pytest.fixture(scope="module")
def ctxs():
    cs = [W.Context(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


def _check_full(buf, ri, g, tag):
    """the joined ReadAll against the oracle's over the whole WAL, every field"""
    o = O.readall(bytes(buf), ri)
    got = (g.status, g.fail_record if g.status not in (O.OK, O.ERR_INDEX_NOT_FOUND) else -1, g.n_records)
    assert got == _want(bytes(buf), ri), (tag, got, _want(bytes(buf), ri))
    if o["status"] == O.OK:
        gd = g.as_dict()
        for k in ("last_crc", "enti", "metadata", "state"):
            assert gd[k] == o[k], (tag, k, gd[k], o[k])
        assert gd["ents"] == o["ents"], tag
    elif o["status"] == O.ERR_INDEX_NOT_FOUND:
        assert g.enti == o["enti"], tag


@pytest.mark.parametrize("n", [2, 3])
def test_multi_inside_file_mutated(ctxs, n):
    rng = random.Random(500 + n)
    resplits = 0
    for i in range(24):
        buf = _wal(rng, n=rng.randrange(60, 300), cuts=rng.randrange(0, 3))
        if i % 4:
            buf = _mutate(rng, buf)
        g, t = W.readall_multi(ctxs[:n], buf, 1)
        _check_full(buf, 1, g, i)
        resplits += t["resplits"]
    assert resplits   # damage at a range edge made some ranges read joined


@pytest.mark.parametrize("n", [2, 3])
def test_multi_by_file_mutated(ctxs, n):
    rng = random.Random(600 + n)
    for i in range(20):
        files = build_files(rng, n * 2, ents=(3, 30))
        blobs = [bytes(b) for b, _ in files]
        if i % 3:
            k = rng.randrange(len(blobs))
            blobs[k] = _mutate(rng, blobs[k])
        if i == 1:   # a middle file ending in a bare length prefix
            blobs[1] += struct.pack("<q", 40)
        buf = b"".join(blobs)
        g, _ = W.readall_multi(ctxs[:n], buf, 0, files=[(len(b), idx) for b, (_, idx) in zip(blobs, files)])
        _check_full(buf, 0, g, i)


def _rich_wal(rng, n_ents, rewinds=False):
    """metadata in every file, HardStates between entries, entries carrying
    unknown fields and a leader change's index rewind: what the stitched
    result has to carry across the ranges"""
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"node-md")
    idx = 1
    for i in range(n_ents):
        if rewinds and i and i % 37 == 0:
            idx = max(1, idx - rng.randrange(1, 4))
        data = rng.randbytes(rng.randrange(0, 400))
        if i % 23 == 5:
            e.encode(2, O.entry_marshal(0, 3, idx, data) + bytes([0x38, i & 0x7F]))
        else:
            e.save_entry(0, 3, idx, data)
        idx += 1
        if i % 17 == 3:
            e.save_state(3, 1, idx - 2)
        if i % 61 == 60:   # a cut: the next file opens with the running CRC and the metadata again
            e.save_crc(e.crc)
            e.encode(1, b"node-md")
    e.encode(3, O.hardstate_marshal(4, 2, idx - 1) + bytes([0x20, 0x05]))
    return e.getvalue()


@pytest.mark.parametrize("n", [2, 3])
def test_multi_by_file_state_unrec_in_entryless_last_file(ctxs, n):
    """ADVICE r05 (medium) on the GPU: by file, the last file holds only
    crcType, metadata and a HardState with XXX_unrecognized (no entry op, so
    its range's own ReadAll is ErrIndexNotFound and keeps no side list); the
    driver's re-read must settle on the whole ReadAll's result -- the HardState
    with its unknown bytes included (round 5: EWAL_E_INVAL after n + 1
    resplits)."""
    from test_split_join import _state_only_last_file
    rng = random.Random(770 + n)
    files = _state_only_last_file(rng, nfiles=12)
    buf = b"".join(b for b, _ in files)
    # whole files grouped so that the driver's byte shares put the entry-less
    # last file alone in the last range: group r opens at the first file
    # boundary at or past r * len / n (ewal_multi_readall's by-file split)
    offs = [0]
    for b, _ in files:
        offs.append(offs[-1] + len(b))
    cut = [0] + [next(i for i in range(len(files)) if offs[i] >= r * len(buf) / n) for r in range(1, n - 1)]
    cut += [len(files) - 1, len(files)]
    groups = [(offs[cut[j + 1]] - offs[cut[j]], files[cut[j]][1]) for j in range(len(cut) - 1)]
    assert len(groups) == n + 0 and groups[-1][0] == len(files[-1][0])
    for ri in (1, 2):
        g, t = W.readall_multi(ctxs[:n], buf, ri, files=groups)
        _check_full(buf, ri, g, ("state_unrec", n, ri))
        assert g.state.XXX_unrecognized == bytes([0x20, 0x05])
        assert t["resplits"] >= 1


@pytest.mark.parametrize("n", [2, 3])
def test_multi_full_result_rich(ctxs, n):
    """metadata, the last HardState (with XXX_unrecognized), ents with
    unknown fields and index rewinds, joined from 2 / 3 ranges inside a file"""
    rng = random.Random(700 + n)
    for i in range(8):
        buf = _rich_wal(rng, rng.randrange(100, 400), rewinds=i % 2 == 1)
        for ri in (1, 7):
            g, _ = W.readall_multi(ctxs[:n], buf, ri)
            _check_full(buf, ri, g, (i, ri))


@pytest.mark.parametrize("n", [2, 3])
def test_multi_device_resident_1gib(ctxs, n):
    """configs[1]-shaped WAL (64 B - 64 KiB entries) of 1 GiB resident in HBM,
    split over n ctxs on device 0 at 16-B aligned frame starts (no copy):
    the joined result equals the faithful oracle's ReadAll over the same bytes
    (verdict, lastCRC, enti, metadata, HardState, the ents digest over every
    entry's fields and Data) and the single-ctx ReadAll exactly (every entry
    descriptor)."""
    import ctypes as C
    from etcd_amd import _lib as L
    buf, nrec = W.synth_wal(1 << 30, 64, 65536, seed=5)
    hb = bytes(buf)
    o = O.readall_digest(hb, 1)
    assert o["status"] == O.OK and o["n_records"] == nrec
    d = ctxs[0].alloc(len(buf) + 64)
    d.upload_ptr(C.addressof((C.c_char * len(buf)).from_buffer(buf)), len(buf))
    try:
        one = W.readall_device(d, len(buf), 1, host_view=memoryview(buf))
        assert one.status == O.OK and one.n_records == nrec
        ne = one.n_ents if hasattr(one, "n_ents") else None
        a1 = (L.EntryDesc * max(1, nrec))()
        k1 = L.lib.ewal_copy_entries(ctxs[0].handle, a1, nrec)
        m = W.Multi(ctxs[:n])
        try:
            plan = m.plan_device(d, len(buf), 1)
            assert all(s % 16 == 0 for s in plan[0][:-1]) and len(set(plan[0])) == n + 1, plan
            g = m.readall_device(d, len(buf), 1, plan=plan)
            assert (g.status, g.n_records, g.last_crc, g.enti) == (o["status"], o["n_records"], o["last_crc"], o["enti"])
            assert g.metadata == o["metadata"]
            assert (g.state.Term, g.state.Vote, g.state.Commit) == o["state"]
            assert (g.status, g.n_records, g.last_crc, g.enti) == (one.status, one.n_records, one.last_crc, one.enti)
            assert g.metadata == one.metadata and g.state == one.state
            assert m.timing()["resplits"] == 0
            a2 = (L.EntryDesc * max(1, nrec))()
            k2 = L.lib.ewal_multi_copy_entries(m._h, a2, nrec)
            assert k1 == k2 == g.n_ents == o["n_ents"] and (ne is None or ne == k1)
            assert O.ent_views_digest(hb, a2, k2) == o["ents_digest"]
            assert C.string_at(a1, k1 * C.sizeof(L.EntryDesc)) == C.string_at(a2, k2 * C.sizeof(L.EntryDesc))
            # and from host bytes (each range staged into its ctx's buffer)
            h = m.readall(buf, 1, with_ents=False)
            assert (h.status, h.n_records, h.last_crc, h.enti, h.metadata) == \
                (one.status, one.n_records, one.last_crc, one.enti, one.metadata)
        finally:
            m.close()
    finally:
        d.free()


def _entry_panic_wal():
    """a WAL whose frame k is an entry record with a wrong stored CRC and an
    Entry.Data length that decodes negative (raft.pb.go:254 panics): the
    whole ReadAll fails its CRC check first (walpb.ErrCRCMismatch)"""
    rng = random.Random(9)
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"md")
    for i in range(1, 40):
        e.save_entry(0, 1, i, rng.randbytes(rng.randrange(10, 300)))
    split = len(e.getvalue())
    e.encode(2, bytes([0x08, 0x00, 0x10, 0x01, 0x18, 40, 0x22]) + b"\xff" * 9 + b"\x01")
    for i in range(41, 60):
        e.save_entry(0, 1, i, rng.randbytes(rng.randrange(10, 300)))
    buf = bytearray(e.getvalue())
    # the crafted frame's stored CRC: flip a bit of its first varint byte (08 02 10 <crc>)
    buf[split + 8 + 3] ^= 0x01
    return bytes(buf), split


def test_join_frame0_entry_decode_after_crc(ctx):
    """range 1 opens (inside a file) on a frame whose Entry
    decode fails; its own read reports that failure at frame 0 (its CRC check
    is deferred), but decoder.decode's Validate runs before mustUnmarshalEntry,
    so the joined verdict is the deferred CRC mismatch -- the oracle's."""
    buf, split = _entry_panic_wal()
    want = _want(buf, 1)
    assert want[0] == O.ERR_RECORD_CRC
    rows, blobs = [], []
    for s, e in ((0, split), (split, len(buf))):
        part = buf[s:e]
        d = ctx.alloc(len(part) + 64)
        d.upload(part)
        g = W.readall_range_device(d, len(part), 1, defer_first=s > 0)
        info = W.range_info(ctx, stream=part)
        d.free()
        if s:   # the range's own verdict is the Entry decode's, at frame 0, after the CRC check
            assert (g.fail_record, info["first_pre_crc"]) == (0, 0) and g.status != O.OK
        r, b = shard.range_row((g.status, g.fail_record, g.n_records, g.last_crc), info, 1, deferred=s > 0)
        rows.append(r)
        blobs.append(b)
    assert shard.join_rows(rows, blobs, 1)[:3] == want


@pytest.mark.parametrize("seed", range(4))
def test_multi_inside_file_tile_spanning_entries(ctxs, seed):
    """the fuzz suite's multi-MiB case (entries spanning whole frame-pass
    tiles, leader changes, mutations) split inside its one file over 2 and 3
    ctxs: the joined ReadAll equals the oracle's"""
    from test_gpu_fuzz import _large_case
    buf, ri = _large_case(40 + seed)
    for n in (2, 3):
        g, _ = W.readall_multi(ctxs[:n], buf, ri)
        _check_full(buf, ri, g, (seed, n))
