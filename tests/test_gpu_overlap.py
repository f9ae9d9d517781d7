"""GPU parity of the overlapped pipeline (round 5, ewal_api.hip ov_launch,
opt-in: EWAL_OPT_OVERLAP): a single WAL of >= 512 MiB is streamed in chunks
on one CU-masked stream while each finished chunk's frame pass runs on the
other CUs, the last chunk's frame pass and the seam pass on the call's own
stream.  Every outcome must be the oracle's ReadAll (wal/wal.go:164-216) --
clean, a corrupt record in the first chunk, in the frame that straddles a
chunk boundary and in the last chunk, a torn tail, an index rewind (the frame
pass's rewind mode), a range of a WAL split inside a file (frame 0's check
deferred) -- and the default (serial) pipeline and the general path
(EWAL_OPT_GENERAL_PATH) must agree."""
import bisect

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from test_gpu_configs import _assert_result, _readall

pytestmark = pytest.mark.gpu

SIZE = 1 << 30   # 1024 tiles of 1 MiB: the default 8 chunks of 128 tiles


@pytest.fixture(scope="module")
def big():
    buf, n = W.synth_wal(SIZE, 64, 65536, seed=21)
    return bytes(buf), n


def _both_paths(ctx, b, ri=1):
    """the overlapped pipeline, the serial one and the general path over the
    same bytes, each against the oracle"""
    o = O.readall_digest(b, ri)
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        try:
            ctx.set_options(overlap=True)
            g = _readall(ctx, d, len(b), ri, memoryview(b))
            _assert_result(ctx, g, o, b)
            for general in (False, True):
                ctx.set_options(general_path=general)
                g2 = _readall(ctx, d, len(b), ri, memoryview(b))
                _assert_result(ctx, g2, o, b)
        finally:
            ctx.set_options()
    finally:
        d.free()
    return g, o


def _frame_at(ctx, b, pos):
    """the frame holding stream byte pos (descriptors of a clean ReadAll)"""
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        r = W.readall_device(d, len(b), 1)
        recs = W.records(ctx, r.n_records)
    finally:
        d.free()
    offs = [x["offset"] for x in recs]
    i = bisect.bisect_right(offs, pos) - 1
    return i, recs[i]


def test_overlap_clean_and_fast_path(ctx, big):
    b, n = big
    g, o = _both_paths(ctx, b)
    assert o["status"] == O.OK and g.n_records == n


@pytest.mark.parametrize("where", ["first_chunk", "chunk_boundary", "last_chunk"])
def test_overlap_corrupt_record(ctx, big, where):
    b, n = big
    pos = {"first_chunk": 5 << 20, "chunk_boundary": 128 << 20, "last_chunk": len(b) - (3 << 20)}[where]
    k, rec = _frame_at(ctx, b, pos)
    bad = bytearray(b)
    bad[rec["data_off"] + rec["data_len"] // 2] ^= 0x5A
    g, o = _both_paths(ctx, bytes(bad))
    assert o["status"] == O.ERR_RECORD_CRC and g.fail_record == k


def test_overlap_torn_tail(ctx, big):
    b, _ = big
    g, o = _both_paths(ctx, b[:-7])
    assert o["status"] == O.ERR_UNEXPECTED_EOF


def test_overlap_rewind_mode(ctx):
    li = []
    buf, _ = W.synth_wal(640 << 20, 64, 65536, seed=22, rewind_per_mille=10, last_index=li)
    g, o = _both_paths(ctx, bytes(buf))
    assert o["status"] == O.OK and o["n_ents"] == li[0]
    # a second call on the same ctx starts in rewind mode (the hint), overlapped too
    d = ctx.alloc(len(buf) + 64)
    try:
        d.upload(bytes(buf))
        ctx.set_options(overlap=True)
        for _ in range(2):
            g2 = _readall(ctx, d, len(buf), 1, memoryview(bytes(buf)))
            _assert_result(ctx, g2, o, bytes(buf))
    finally:
        ctx.set_options()
        d.free()


def test_overlap_deferred_range(ctx, big):
    """a >= 512 MiB range of a WAL split inside a file: frame 0's check is the
    caller's (EWAL_RANGE_DEFER_FIRST); its range info must match the general
    path's"""
    b, _ = big
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        start, ri = W.range_probe(d, len(b), 300 << 20, 1 << 20)
    finally:
        d.free()
    assert start > 0 and ri > 1
    part = b[start:]
    d = ctx.alloc(len(part) + 64)
    try:
        d.upload(part)
        infos = []
        for general, overlap in ((False, True), (False, False), (True, False)):
            ctx.set_options(general_path=general, overlap=overlap)
            try:
                g = W.readall_range_device(d, len(part), ri, defer_first=True)
                infos.append(((g.status, g.n_records, g.last_crc, g.enti), W.range_info(ctx, stream=part)))
            finally:
                ctx.set_options()
        assert infos[0] == infos[1] == infos[2]
        assert infos[0][0][0] == O.OK
    finally:
        d.free()
