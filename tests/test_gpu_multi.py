"""ONE WAL split over several contexts in one process (ewal_readall_multi,
VERDICT r03 #3): one host thread per ctx -- here 2 and 3 ctxs on device 0 --
each reading its range (whole files, or a range opening at a frame-start
candidate inside a file with frame 0's check deferred), and ReadAll's
cross-range rules joined in the C ABI (ewal_split_verdict, the join
etcd_amd/shard.py also calls after its torch.distributed exchange).  The
joined verdict must be the oracle's ReadAll over the whole WAL, on clean and
on damaged WALs (test_gpu_fuzz's mutations), and on the two cases ADVICE r03
found in the Python join: a range whose frame 0 fails its Entry decode (that
comes after decoder.decode's CRC check, so the deferred CRC check wins) and a
file ending in a bare length prefix (io.EOF for the range alone)."""
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


@pytest.mark.parametrize("n", [2, 3])
def test_multi_inside_file_mutated(ctxs, n):
    rng = random.Random(500 + n)
    resplits = 0
    for i in range(24):
        buf = _wal(rng, n=rng.randrange(60, 300), cuts=rng.randrange(0, 3))
        if i % 4:
            buf = _mutate(rng, buf)
        g = W.readall_multi(ctxs[:n], buf, 1)
        assert g[:3] == _want(buf, 1), (i, g, _want(buf, 1))
        if g[0] == O.OK:
            assert g[3] == O.readall(buf, 1)["last_crc"]
        resplits += g[5]
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
        g = W.readall_multi(ctxs[:n], buf, 0, files=[(len(b), idx) for b, (_, idx) in zip(blobs, files)])
        assert g[:3] == _want(buf, 0), (i, g, _want(buf, 0))


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
