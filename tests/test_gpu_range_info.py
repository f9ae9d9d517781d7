"""ewal_copy_range_info after a ReadAll the frame pass decided (round 5:
k_range_info_fr reads the pass's reductions -- the frames the info names, their
ordinals, frame 0's crc32.Update(0, Data) -- instead of rebuilding every
frame's descriptor): field by field the info the descriptors give
(k_range_info over the rebuilt descriptors, forced by ewal_copy_records), and
the oracle's decoders (test_split_wal.oracle_range_info) where every frame is
framable.  Reference: what one range of a split WAL contributes to ReadAll's
cross-file rules, wal/wal.go:164-216 (crc seam 184-190, metadata 175-181,
ents 170-174, state 182)."""
import random

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from test_split_wal import _cases, oracle_range_info

pytestmark = pytest.mark.gpu


def _both(ctx, g, buf):
    """(the fused info, the info from the rebuilt descriptors) of the last ReadAll"""
    fused = W.range_info(ctx, stream=buf)
    W.records(ctx, 1)                       # rebuilds the descriptors (rd_valid from here on)
    rebuilt = W.range_info(ctx, stream=buf)
    return fused, rebuilt


def test_range_info_fused_split_cases(ctx):
    fast = 0
    for world in (2, 3):
        for allb, rig, ranges in _cases(random.Random(17 + world), world):
            for buf, ri in ranges + [(allb, rig)]:
                if not buf:
                    continue
                g = W.readall_bytes(buf, ri, ctx, with_ents=False)
                fast += bool(g.flags & L.FLAG_FAST_PATH)
                fused, rebuilt = _both(ctx, g, buf)
                assert fused == rebuilt, (fused, rebuilt)
                if g.status == O.OK:
                    assert fused == oracle_range_info(buf, ri)
    assert fast > 0   # the frame pass decided some of them (the path under test ran)


@pytest.mark.parametrize("size,lo,hi", [(8 << 20, 64, 4096), (24 << 20, 16, 65536)])
def test_range_info_fused_deferred_ranges(ctx, size, lo, hi):
    """ranges of a WAL split inside a file (frame 0's check deferred: its
    crc32.Update(0, Data) from the frame pass), cut at several offsets"""
    buf, n = W.synth_wal(size, lo, hi, seed=31)
    b = bytes(buf)
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        cuts = []
        for frac in (0.1, 0.37, 0.5, 0.83, 0.999):
            p, idx = W.range_probe(d, len(b), int(len(b) * frac) & ~7, 1 << 20)
            if p > 0:
                cuts.append((p, idx))
    finally:
        d.free()
    assert cuts
    for p, idx in cuts:
        part = b[p:]
        d = ctx.alloc(len(part) + 64)
        try:
            d.upload(part)
            g = W.readall_range_device(d, len(part), idx, defer_first=True)
            assert g.status == O.OK and g.flags & L.FLAG_FAST_PATH
            fused, rebuilt = _both(ctx, g, part)
        finally:
            d.free()
        assert fused == rebuilt
        assert fused == oracle_range_info(part, idx)   # first_u0 = crc32.Update(0, frame 0's Data)


def test_range_info_fused_entries_below_ri_and_rewinds(ctx):
    """an entry below ri (no op) and index rewinds: the descriptors decide"""
    # ri inside the WAL: the first entries are below it
    buf, n = W.synth_wal(4 << 20, 64, 2048, seed=32)
    b = bytes(buf)
    for ri in (1, 5, 200):
        g = W.readall_bytes(b, ri, ctx, with_ents=False)
        fused, rebuilt = _both(ctx, g, b)
        assert fused == rebuilt == oracle_range_info(b, ri)
    # index rewinds (the rewind-mode pass on the second call)
    li = []
    buf, _ = W.synth_wal(6 << 20, 64, 2048, seed=33, rewind_per_mille=20, last_index=li)
    b = bytes(buf)
    for _ in range(2):
        g = W.readall_bytes(b, 1, ctx, with_ents=False)
        fused, rebuilt = _both(ctx, g, b)
        assert fused == rebuilt == oracle_range_info(b, 1)


def test_range_info_fused_failures(ctx):
    """a corrupt record, a torn tail: the info covers the chain's frames either way"""
    buf, n = W.synth_wal(4 << 20, 64, 4096, seed=34)
    b = bytearray(buf)
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(bytes(b))
        W.readall_device(d, len(b), 1)
        recs = W.records(ctx, n)
    finally:
        d.free()
    bad = bytearray(b)
    r = recs[len(recs) // 2]
    bad[r["data_off"] + r["data_len"] // 2] ^= 0x40
    for x in (bytes(bad), bytes(b[:-9])):
        g = W.readall_bytes(x, 1, ctx, with_ents=False)
        assert g.status != O.OK
        fused, rebuilt = _both(ctx, g, x)
        assert fused == rebuilt
