"""GPU parity of the frame pass's prefix at every frame-start offset inside a
super-piece (round 6: the tail as the lin of the load's 128-B block -- 64-B
with vh[] -- with the other bytes masked, moved into place by table shifts;
`prefix_near_tail`, wal_kernels.hip).  A WAL of 1..200-byte records puts
frame starts on all 256 offsets of a 256-B super-piece (asserted), so both
directions, the 16-B chunk edges, the mid point and the unit's last
super-piece all occur; corrupt records at chosen offsets must fail where the
oracle's ReadAll fails (wal/wal.go:164-216: status, failing frame, offset),
and streams cut so that the last frame starts in the upper half of a partial
last super-piece take the general prefix (no boundary above)."""
import pytest

from oracle import oracle as O
from etcd_amd import wal as W
from test_gpu_configs import _assert_result
from test_gpu_vh import _dev_readall

pytestmark = pytest.mark.gpu

# offsets inside a super-piece: both ends, the 16-B chunk edges around the
# 64-B and 128-B points (vh[]'s and the 256-B form's direction switches)
RESIDUES = [0, 1, 3, 15, 16, 17, 47, 63, 64, 65, 79, 111, 127, 128, 129, 143, 175, 191, 192, 193, 223, 239, 254,
            255]


def _frame_starts(b):
    """frame start offsets by the reference's framing (wal/decoder.go:79-83:
    an int64 little-endian length, then that many record bytes)"""
    p, out = 0, []
    while p + 8 <= len(b):
        n = int.from_bytes(b[p:p + 8], "little", signed=True)
        if n <= 0 or p + 8 + n > len(b):
            break
        out.append(p)
        p += 8 + n
    return out


@pytest.fixture(scope="module")
def dense_wal():
    buf, _ = W.synth_wal(3 << 20, 1, 200, seed=77)
    b = bytes(buf)
    starts = _frame_starts(b)
    assert starts and starts[-1] < len(b)
    return b, starts


def test_frame_starts_cover_every_offset(ctx, dense_wal):
    b, starts = dense_wal
    assert {p % 256 for p in starts} == set(range(256))
    o = O.readall_digest(b, 1)
    assert o["status"] == O.OK and o["n_records"] == len(starts)
    for vh in (True, False):
        _assert_result(ctx, _dev_readall(ctx, b, 1, vh), o, b)


@pytest.mark.parametrize("r", RESIDUES)
def test_corrupt_record_at_offset(ctx, dense_wal, r):
    b, starts = dense_wal
    # a frame well inside the stream whose start sits at offset r of its super-piece
    k = next(i for i, p in enumerate(starts) if i > 100 and p % 256 == r)
    end = starts[k + 1] if k + 1 < len(starts) else len(b)
    x = bytearray(b)
    x[end - 1] ^= 0x5A   # the record's last byte: its Data, the head stays canonical
    x = bytes(x)
    o = O.readall_digest(x, 1)
    assert o["status"] != O.OK
    for vh in (True, False):
        _assert_result(ctx, _dev_readall(ctx, x, 1, vh), o, x)


@pytest.mark.parametrize("blk,lo,hi", [(256, 129, 170), (256, 170, 210), (256, 210, 256), (128, 65, 100),
                                        (128, 100, 128)])
def test_last_frame_in_partial_last_block(ctx, dense_wal, blk, lo, hi):
    b, starts = dense_wal
    # cut at a frame end so that the last frame starts in [lo, hi) of a
    # super-piece (blk 256) or a 128-B half (vh[]) the stream does not complete
    for i in range(len(starts) - 2, 200, -1):
        p, e = starts[i], starts[i + 1]
        if lo <= p % blk < hi and e - (p & ~(blk - 1)) < blk:
            break
    else:
        pytest.skip("no such frame")
    x = b[:e]
    o = O.readall_digest(x, 1)
    assert o["status"] == O.OK
    for vh in (True, False):
        _assert_result(ctx, _dev_readall(ctx, x, 1, vh), o, x)


@pytest.mark.parametrize("seed", range(2))
def test_records_over_one_mib(ctx, seed):
    """Data longer than 2^20 bytes: the checks' S_dlen past the table rounds
    and the seam pass's shifts past its hex-digit tables (frame_kernels.hip
    seam_shift) take the powers-of-two remainder; clean and with one corrupt
    record, against the oracle."""
    buf, n = W.synth_wal(48 << 20, 1 << 20, 3 << 20, seed=880 + seed)
    b = bytes(buf)
    assert n >= 8
    for x in (b, bytes(W.synth_wal(48 << 20, 1 << 20, 3 << 20, seed=880 + seed, corrupt_record=n // 2)[0])):
        o = O.readall_digest(x, 1)
        assert (o["status"] == O.OK) == (x is b)
        for vh in (True, False):
            _assert_result(ctx, _dev_readall(ctx, x, 1, vh), o, x)
