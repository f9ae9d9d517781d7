"""Split byte fields on the GPU: a walpb.Record whose Data, or a raftpb.Entry
whose Data, is repeated with several non-empty segments.  Go's Unmarshal
appends them (`m.Data = append(m.Data, ...)`, wal/walpb/record.pb.go:112,
raft/raftpb/raft.pb.go:254), so the Record's CRC, the metadata, the Entry /
HardState decoded from it and the Entry's Data are all the concatenation.
etcd's encoder never writes this; a crafted WAL can.  The engine gathers the
concatenations into a device side arena (ewal_copy_split_bytes) and must
match the oracle exactly -- never EWAL_UNSUPPORTED_ENCODING."""
import random
import struct

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def _uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _bytes_field(fnum, b):
    return _uvarint(fnum << 3 | 2) + _uvarint(len(b)) + b


class SplitWal:
    """The reference encoder's framing (wal/encoder.go:25-37) with Record.Data
    given as segments (the running CRC over their concatenation)."""

    def __init__(self, prev=0):
        self.crc = prev
        self.out = bytearray()

    def record(self, type_, segs, crc_override=None):
        data = b"".join(segs)
        if type_ != 4:
            self.crc = O.crc32_update(self.crc, data)
        crc = self.crc if crc_override is None else crc_override
        body = bytes([0x08]) + _uvarint(type_) + bytes([0x10]) + _uvarint(crc)
        for s in segs:
            body += _bytes_field(3, s)
        self.out += struct.pack("<q", len(body)) + body

    def plain(self, type_, data):
        self.record(type_, [data] if data else [])

    def entry(self, term, index, data, nseg=1, rng=None):
        b = O.entry_marshal(0, term, index, data)
        self.record(2, _cut(b, nseg, rng))

    def getvalue(self):
        return bytes(self.out)


def _cut(b, nseg, rng):
    """b in nseg non-empty pieces at random points (mid-varint included)."""
    if nseg <= 1 or len(b) < nseg:
        return [b]
    pts = sorted((rng or random.Random(len(b))).sample(range(1, len(b)), nseg - 1))
    return [b[i:j] for i, j in zip([0] + pts, pts + [len(b)])]


def _entry_split_data(term, index, segs, etype=0, unk=b""):
    """An Entry whose Data field (4) is repeated: one occurrence per segment."""
    b = bytes([0x08]) + _uvarint(etype) + bytes([0x10]) + _uvarint(term) + bytes([0x18]) + _uvarint(index)
    for s in segs:
        b += _bytes_field(4, s)
    return b + unk


def test_split_record_data_all_types(ctx):
    rng = random.Random(7)
    w = SplitWal()
    w.record(4, [])
    w.record(1, [b"meta", b"", b"data"])                 # split metadata (an empty repeat in between)
    w.record(3, _cut(O.hardstate_marshal(1, 2, 0), 3, rng))
    for i in range(1, 40):
        w.entry(1, i, bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300))),
                nseg=rng.choice([1, 1, 2, 3, 5]), rng=rng)
    w.record(3, _cut(O.hardstate_marshal(2, 1, 30), 2, rng))
    o, g = assert_parity(ctx, w.getvalue(), 1)
    assert o["status"] == O.OK and g["metadata"] == b"metadata" and len(g["ents"]) == 39
    r = W.readall_bytes(w.getvalue(), 1, ctx)
    assert r.flags & L.FLAG_METADATA_SPLIT


def test_split_entry_data(ctx):
    rng = random.Random(8)
    w = SplitWal()
    w.record(4, [])
    w.plain(1, b"m")
    w.plain(2, _entry_split_data(1, 1, [b"ab", b"cd", b"", b"ef"]))              # Entry.Data split in a plain record
    w.record(2, _cut(_entry_split_data(1, 2, [b"x" * 100, b"y" * 50]), 3, rng))  # ... inside a split record too
    w.plain(2, _entry_split_data(1, 3, [b"only"]))                              # one segment: a stream view
    w.plain(2, _entry_split_data(1, 4, [b"", b"z"]))                            # empty first repeat
    w.plain(2, _entry_split_data(1, 5, [b"u", b"v"], unk=bytes([0x38, 0x05])))  # + XXX_unrecognized
    o, g = assert_parity(ctx, w.getvalue(), 1)
    assert o["status"] == O.OK
    assert [e["data"] for e in g["ents"]] == [b"abcdef", b"x" * 100 + b"y" * 50, b"only", b"z", b"uv"]
    assert g["ents"][4]["unrec"] == bytes([0x38, 0x05])


def test_split_unknown_fields_in_concatenation(ctx):
    # the Entry / HardState decoded from a concatenation carry XXX_unrecognized
    rng = random.Random(9)
    w = SplitWal()
    w.record(4, [])
    w.plain(1, b"m")
    w.record(2, _cut(O.entry_marshal(0, 1, 1, b"payload") + bytes([0x38, 0x07]), 3, rng))
    w.record(3, _cut(O.hardstate_marshal(1, 1, 1) + bytes([0x20, 0x09]), 2, rng))
    o, g = assert_parity(ctx, w.getvalue(), 1)
    assert o["status"] == O.OK
    assert g["ents"][0]["unrec"] == bytes([0x38, 0x07]) and g["state"]["unrec"] == bytes([0x20, 0x09])


def test_split_failures(ctx):
    rng = random.Random(10)
    base = SplitWal()
    base.record(4, [])
    base.plain(1, b"mm")
    for i in range(1, 5):
        base.entry(1, i, b"q" * 20)
    pre = base.getvalue()
    # a split record whose stored CRC is wrong: walpb.ErrCRCMismatch there
    w = SplitWal(base.crc)
    w.out += pre
    w.record(2, _cut(O.entry_marshal(0, 1, 5, b"abc"), 2, rng), crc_override=12345)
    assert_parity(ctx, w.getvalue(), 1)
    # a split record whose concatenation is no valid Entry: mustUnmarshalEntry panics
    w = SplitWal(base.crc)
    w.out += pre
    w.record(2, [bytes([0x08]), bytes([0x80])])   # varint runs off the end
    o, _ = assert_parity(ctx, w.getvalue(), 1)
    assert o["status"] == O.PANIC_ENTRY
    # a split metadata that differs from the first: ErrMetadataConflict; equal: fine
    for tail, want in ((b"mx", O.ERR_METADATA_CONFLICT), (b"mm", O.OK)):
        w = SplitWal(base.crc)
        w.out += pre
        w.record(1, [tail[:1], tail[1:]])
        w.entry(1, 5, b"r")
        o, _ = assert_parity(ctx, w.getvalue(), 1)
        assert o["status"] == want
    # an index gap on an entry decoded from a concatenation
    w = SplitWal(base.crc)
    w.out += pre
    w.entry(1, 7, b"gap", nseg=3, rng=rng)
    o, _ = assert_parity(ctx, w.getvalue(), 1)
    assert o["status"] == O.PANIC_INDEX_GAP


def test_split_large_grows_the_arena(ctx):
    # concatenations beyond the arena's first size (1 MiB): the call grows it
    # and runs again -- still exact
    rng = random.Random(11)
    w = SplitWal()
    w.record(4, [])
    w.plain(1, b"m")
    big = bytes(rng.getrandbits(8) for _ in range(700_000))
    w.plain(2, _entry_split_data(1, 1, [big[:300_000], big[300_000:]]))
    w.entry(1, 2, big[::-1], nseg=4, rng=rng)
    w.entry(1, 3, b"after")
    o, g = assert_parity(ctx, w.getvalue(), 1)
    assert o["status"] == O.OK and g["ents"][0]["data"] == big and g["ents"][1]["data"] == big[::-1]


def test_split_batch_shard_replayed_alone(ctx):
    rng = random.Random(12)
    w = SplitWal()
    w.record(4, [])
    w.record(1, [b"me", b"ta"])
    for i in range(1, 20):
        w.entry(1, i, bytes([i]) * i, nseg=2 if i % 3 == 0 else 1, rng=rng)
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"plain")
    for i in range(1, 30):
        e.save_entry(0, 1, i, b"p" * i)
    shards = [w.getvalue(), e.getvalue(), w.getvalue()]
    res = W.readall_batch_bytes(shards, [1, 1, 1], ctx)
    for s, r in zip(shards, res):
        o = O.readall(s, 1)
        assert r.status == o["status"] == O.OK
        assert r.metadata == o["metadata"]
        assert [(x.Index, x.Term, x.Data) for x in r.ents] == [(x["index"], x["term"], x["data"]) for x in o["ents"]]
    assert res[0].flags & L.FLAG_SHARD_FALLBACK and res[2].flags & L.FLAG_SHARD_FALLBACK


@pytest.mark.parametrize("seed", range(6))
def test_split_random(ctx, seed):
    rng = random.Random(500 + seed)
    w = SplitWal()
    w.record(4, [])
    w.record(1, _cut(b"metadata-" + bytes([seed]), rng.choice([1, 2, 3]), rng))
    idx = 1
    for _ in range(rng.randrange(5, 80)):
        k = rng.random()
        if k < 0.1:
            w.record(3, _cut(O.hardstate_marshal(rng.randrange(1, 9), 1, idx), rng.choice([1, 2]), rng))
        elif k < 0.2:
            w.plain(2, _entry_split_data(1, idx, [bytes([idx & 0xff]) * rng.randrange(1, 50)
                                                  for _ in range(rng.randrange(2, 5))]))
            idx += 1
        else:
            w.entry(1, idx, bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 500))),
                    nseg=rng.choice([1, 2, 4]), rng=rng)
            idx += 1
    buf = bytearray(w.getvalue())
    if seed % 3 == 2:   # a flipped byte somewhere
        buf[rng.randrange(len(buf))] ^= 1 << rng.randrange(8)
    o, g = assert_parity(ctx, bytes(buf), 1)
    assert g["status"] != L.UNSUPPORTED_ENCODING
