"""GPU parity of the framing paths the candidate filter does not cover.

* Every single-bit corruption of the reference's `infoRecord`
  (wal/record_test.go:31-32) and of a small WAL (crc + metadata + state +
  3 entries): the error identity must equal the oracle's (decoder.decode,
  wal/decoder.go:28-47; Record.Unmarshal, record.pb.go:43-136) -- the frame
  the corruption turns into a non-candidate is decoded by k_walk on the GPU,
  never reported as EWAL_UNSUPPORTED_ENCODING.
* Valid frames in non-canonical encodings (fields out of order, non-minimal
  varints, unknown fields) in the middle of a WAL: the chain continues
  through them (k_walk, then pointer jumping resumes at the next candidate).
* Entries whose Data embed well-formed frames (false candidates) force the
  pointer-jumping framing (n_runs > 1) at >= 64 MiB, single and batched.
"""
import random
import struct

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from test_gpu_parity import INFO, assert_parity, build_wal

pytestmark = pytest.mark.gpu


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def nc_record(type_, crc, data, style):
    """A walpb.Record in a non-canonical byte layout Record.Unmarshal accepts
    (record.pb.go:43-136); data None == nil."""
    d = b"" if data is None else b"\x1a" + _varint(len(data)) + data
    if style == "crc_first":
        return b"\x10" + _varint(crc) + b"\x08" + _varint(type_) + d
    if style == "long_type":          # type as a 2-byte varint (non-minimal)
        return b"\x08" + bytes([0x80 | type_, 0x00]) + b"\x10" + _varint(crc) + d
    if style == "unknown_first":      # field 5 varint first: Skip -> XXX_unrecognized
        return b"\x28\x07\x08" + _varint(type_) + b"\x10" + _varint(crc) + d
    if style == "data_first":
        return d + b"\x08" + _varint(type_) + b"\x10" + _varint(crc)
    raise ValueError(style)


class MixedWal:
    """encoder.encode (wal/encoder.go:25-37) with some frames written in a
    non-canonical layout; the chained CRC is the reference's either way."""

    def __init__(self):
        self.buf = bytearray()
        self.crc = 0

    def canonical(self, type_, data):
        e = O.WalEncoder(self.crc)
        e.encode(type_, data)
        self.buf += e.getvalue()
        self.crc = e.crc

    def noncanonical(self, type_, data, style):
        if type_ != 4:
            self.crc = O.crc32_update(self.crc, data or b"")
        body = nc_record(type_, self.crc, data, style)
        self.buf += struct.pack("<q", len(body)) + body

    def entry(self, index, data, style=None):
        e = O.entry_marshal(0, 1, index, data)
        if style:
            self.noncanonical(2, e, style)
        else:
            self.canonical(2, e)


def small_wal():
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"md")
    e.save_state(1, 2, 1)
    for i in range(3):
        e.save_entry(0, 1, i + 1, bytes([0x41 + i]) * (i + 2))
    return e.getvalue()


@pytest.mark.parametrize("name", ["info", "small_wal"])
def test_every_bit_flip(ctx, name):
    base = INFO if name == "info" else small_wal()
    ri = 0 if name == "info" else 1
    seen = {}
    for p in range(len(base)):
        for b in range(8):
            w = bytearray(base)
            w[p] ^= 1 << b
            o, g = assert_parity(ctx, w, ri)
            assert g["status"] != L.UNSUPPORTED_ENCODING
            seen[o["status"]] = seen.get(o["status"], 0) + 1
    # the flips reach many error classes, each decided exactly
    assert len(seen) >= 4, seen


def test_every_byte_value_in_record_head(ctx):
    """Each byte of the first entry frame's head (length prefix + Record
    tags) set to every value 0..255."""
    base = small_wal()
    offs = O.chain_crcs(base)[1]
    head = offs[3]            # crc, metadata, state, entry 1
    for p in range(head, head + 14):
        for v in range(256):
            w = bytearray(base)
            w[p] = v
            o, g = assert_parity(ctx, w, 1, check_chain=False)
            assert g["status"] != L.UNSUPPORTED_ENCODING


@pytest.mark.parametrize("style", ["crc_first", "long_type", "unknown_first", "data_first"])
def test_noncanonical_frames_mid_wal(ctx, style):
    rng = random.Random(sum(map(ord, style)))
    m = MixedWal()
    m.canonical(4, None)
    m.noncanonical(1, b"metadata", style)          # a non-canonical metadata record
    idx = 1
    for seg in range(6):
        for _ in range(rng.randrange(1, 40)):
            m.entry(idx, rng.randbytes(rng.randrange(0, 3000)))
            idx += 1
        for _ in range(rng.randrange(1, 3)):      # runs of non-canonical frames between candidate runs
            m.entry(idx, rng.randbytes(rng.randrange(0, 500)), style)
            idx += 1
    m.noncanonical(3, O.hardstate_marshal(3, 1, idx - 1), style)
    o, g = assert_parity(ctx, m.buf, 1)
    assert o["status"] == O.OK and g["n_records"] == o["n_records"]
    # a corruption after the non-canonical frames is still found exactly
    bad = bytearray(m.buf)
    bad[len(bad) * 3 // 4] ^= 0x08
    assert_parity(ctx, bad, 1)
    # ... and a WAL that ENDS in non-canonical frames / starts with one
    m2 = MixedWal()
    m2.noncanonical(4, None, style)
    m2.canonical(1, b"m")
    m2.entry(1, b"x" * 10)
    m2.entry(2, b"y" * 10, style)
    assert_parity(ctx, m2.buf, 1)
    assert_parity(ctx, m2.buf[:-1], 1)


@pytest.mark.parametrize("style", ["crc_first", "long_type", "data_first"])
def test_noncanonical_frames_in_units_without_candidates(ctx, style):
    """Large non-canonical frames (k_walk) whose frame and data starts lie in
    4 KiB units holding no frame-start candidate: the stream pass writes no
    super-piece lins there, so P comes from the unit start (prefix_slow).
    A corruption inside such a frame's Data is found at the same frame."""
    rng = random.Random(7 + len(style))
    m = MixedWal()
    m.canonical(4, None)
    m.canonical(1, b"metadata")
    idx = 1
    walked = []
    for seg in range(4):
        for _ in range(3):
            m.entry(idx, rng.randbytes(rng.randrange(5000, 14000)))
            idx += 1
        for _ in range(2):
            walked.append((len(m.buf), rng.randrange(6000, 11000)))
            m.entry(idx, rng.randbytes(walked[-1][1]), style)
            idx += 1
    m.canonical(3, O.hardstate_marshal(1, 1, idx - 1))
    o, g = assert_parity(ctx, m.buf, 1)
    assert o["status"] == O.OK and g["n_records"] == o["n_records"]
    for at, n in walked[1::3]:
        bad = bytearray(m.buf)
        bad[at + 40 + n // 2] ^= 0x20        # inside the walked frame's Data
        o, g = assert_parity(ctx, bad, 1)
        assert o["status"] == O.ERR_RECORD_CRC


def test_noncanonical_entry_payload_types(ctx):
    """A non-canonical walked frame whose payload fails mustUnmarshalEntry /
    has an unexpected type / fails its CRC: ReadAll stops at it."""
    for typ, data in ((2, b"\x08"), (3, b"\x0a\x00"), (7, b"zz"), (2, O.entry_marshal(0, 1, 1, b"a"))):
        m = MixedWal()
        m.canonical(4, None)
        m.canonical(1, b"m")
        at = len(m.buf)
        m.noncanonical(typ, data, "crc_first")
        m.entry(2, b"tail")
        assert_parity(ctx, m.buf, 1)
        bad = bytearray(m.buf)
        bad[at + 9] ^= 0x01       # the walked frame's stored CRC (first byte after its 10 tag)
        assert_parity(ctx, bad, 1)


def _false_candidate_wal(rng, target, embed_every=7):
    """Entries whose Data embed well-formed frames (int64 length + canonical
    Record head) -- candidates that are not on the frame chain."""
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"metadata")
    i = 1
    size = 0
    while size < target:
        n = rng.randrange(64, 8192)
        d = bytearray(rng.randbytes(n))
        if i % embed_every == 0:
            inner = O.record_marshal(2, rng.getrandbits(32), rng.randbytes(rng.randrange(0, 40)))
            fr = struct.pack("<q", len(inner)) + inner
            at = rng.randrange(0, max(1, n - len(fr)))
            d[at:at + len(fr)] = fr
            if i % (3 * embed_every) == 0:      # a chain of two false candidates
                at2 = at + len(fr)
                if at2 + len(fr) <= n:
                    d[at2:at2 + len(fr)] = fr
        e.save_entry(0, 1, i, bytes(d))
        size += n + 30
        i += 1
    return e.getvalue(), i - 1


def test_pointer_jumping_64mib(ctx):
    rng = random.Random(64)
    w, n_ent = _false_candidate_wal(rng, 64 << 20)
    g = W.readall_bytes(w, 1, ctx)
    assert g.n_runs > 1, g.n_runs          # the speculative path declined: pointer jumping framed it
    assert g.n_candidates > g.n_records
    o, gd = assert_parity(ctx, w, 1, check_chain=False)
    assert o["status"] == O.OK and len(gd["ents"]) == n_ent
    # a corrupt record in the middle, found exactly through the same path
    offs = O.chain_crcs(w, cap=n_ent + 16)[1]
    k = len(offs) * 2 // 3
    bad = bytearray(w)
    bad[offs[k] + 40] ^= 0x01
    assert_parity(ctx, bad, 1, check_chain=False)
    # batched: the batch declines its fast path and each shard is exact
    small, _ = _false_candidate_wal(rng, 4 << 20, embed_every=3)
    clean = build_wal(rng, 50, 3000)
    res = W.readall_batch_bytes([clean, small, bytes(bad), clean], [0, 1, 1, 0], ctx)
    for buf, ri, r in zip([clean, small, bytes(bad), clean], [0, 1, 1, 0], res):
        ob = O.readall(buf, ri)
        assert (r.status, r.fail_record) == (ob["status"], ob["fail_record"])
        if ob["status"] == O.OK:
            assert (r.n_records, r.last_crc, r.enti) == (ob["n_records"], ob["last_crc"], ob["enti"])


def test_entries_beyond_the_ternary_shift_span(ctx):
    """Entries whose Data is 170-600 KB long: the frame pass applies S_n
    from LDS nibble tables for n below 2^20 and from the global byte tables
    above; every chained CRC and a corruption inside such an entry must
    match the oracle (record.pb.go Data, pkg/crc chaining)."""
    rng = random.Random(11)
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"metadata")
    sizes = [177147 - 40, 177147, 177147 + 5, 200000, 354294, 600000, 3, 65536, 531441]
    for i, n in enumerate(sizes):
        e.save_entry(0, 1, i + 1, rng.randbytes(n))
    buf = e.getvalue()
    o, g = assert_parity(ctx, buf, 1)
    assert o["status"] == O.OK and g["n_records"] == o["n_records"]
    bad = bytearray(buf)
    bad[len(bad) * 2 // 3] ^= 0x01
    o, g = assert_parity(ctx, bad, 1)
    assert o["status"] != O.OK


@pytest.mark.parametrize("tail", [struct.pack("<q", 3) + b"\x00\x01\x02",          # round 4's r04b shape
                                  struct.pack("<q", 4) + b"\x08\x01\x10\x00",      # a whole frame, canonical head
                                  struct.pack("<q", 12) + b"\x10\x05\x08\x02" + bytes(8),
                                  struct.pack("<q", 3) + b"\x00\x01",              # torn: 2 of 3 bytes
                                  struct.pack("<q", 0)])                            # zero length, nothing after
def test_single_wal_trailing_frame_that_fits(ctx, tail):
    """The single-WAL form of test_gpu_batch's t3 shard: a WAL ending in a
    length prefix whose frame fits in the bytes left (decoder.decode then
    Unmarshals it, wal/decoder.go:30-47).  The frame pass declines such a
    terminal (fc.rare 128) and the general path walks it; both option
    settings must give the oracle's verdict, never an infrastructure error."""
    rng = random.Random(len(tail) * 7 + (tail[-1] if tail[8:] else 5))
    base = build_wal(rng, 40, 700, big_terms=False)
    for general in (False, True):
        ctx.set_options(general_path=general)
        try:
            assert_parity(ctx, base + tail, 0, check_chain=False)
            # and behind a WAL long enough for the 64 KiB / 1 MiB tile sizes
            big = build_wal(rng, 1500, 3000, big_terms=False)
            assert_parity(ctx, big + tail, 0, check_chain=False)
        finally:
            ctx.set_options(general_path=False)
