"""GPU parity of the frame pass's 128-B prefixes (round 5, EWAL_OPT_VH_ON /
the record-dense default): the stream pass also stores the lin of every
super-piece's first 128-B half (vh[]), and every frame start's prefix is taken
from the nearest 128-B boundary -- forward over <= 64 bytes, or back over
<= 64 with the inverse shifts.  Every outcome must be the oracle's ReadAll
(wal/wal.go:164-216: status, failing frame and offset, lastCRC, ents, state,
metadata) with the option on, off and automatic, over the frame positions
that hit every case: both halves of a super-piece, both directions, the mid
boundary, the unit's last super-piece (the next unit's start), the stream's
last partial block, corrupt records, torn tails, mutations, index rewinds and
a range whose frame 0 is deferred."""
import random

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from test_gpu_configs import _assert_result, _readall
from test_gpu_fuzz import _mutate
from test_gpu_parity import assert_parity, build_wal

pytestmark = pytest.mark.gpu


def _dev_readall(ctx, b, ri, vh):
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        ctx.set_options(vh=vh)
        try:
            return _readall(ctx, d, len(b), ri, memoryview(b))
        finally:
            ctx.set_options()
    finally:
        d.free()


@pytest.mark.parametrize("size,lo,hi,seed", [(8 << 20, 256, 256, 41), (6 << 20, 16, 512, 42),
                                             (12 << 20, 64, 4096, 43), (3 << 20, 1, 200, 44),
                                             (20 << 20, 100, 1500, 45)])
def test_vh_shapes_against_oracle(ctx, size, lo, hi, seed):
    buf, n = W.synth_wal(size, lo, hi, seed=seed)
    b = bytes(buf)
    o = O.readall_digest(b, 1)
    assert o["status"] == O.OK
    for vh in (True, False, None):
        g = _dev_readall(ctx, b, 1, vh)
        assert g.flags & L.FLAG_FAST_PATH
        _assert_result(ctx, g, o, b)


@pytest.mark.parametrize("seed", range(4))
def test_vh_corrupt_and_torn(ctx, seed):
    rng = random.Random(500 + seed)
    buf, n = W.synth_wal(4 << 20, 32, 700, seed=60 + seed, corrupt_record=rng.randrange(1, 2000))
    b = bytes(buf)
    for x in (b, b[:-rng.randrange(1, 300)]):
        o = O.readall_digest(x, 1)
        assert o["status"] != O.OK or x is not b
        for vh in (True, False):
            _assert_result(ctx, _dev_readall(ctx, x, 1, vh), o, x)


@pytest.mark.parametrize("block", range(4))
def test_vh_mutated_wals(ctx, block):
    rng = random.Random(8300 + block)
    ctx.set_options(vh=True)
    try:
        for _ in range(40):
            w = build_wal(rng, rng.randrange(3, 90), rng.choice([40, 300, 5000]), cuts=rng.randrange(0, 3),
                          big_terms=rng.random() < 0.3)
            assert_parity(ctx, _mutate(rng, w), rng.choice([0, 1, 3]))
        for seed in range(3):   # multi-MiB, record-dense, damaged far from byte 0
            buf, _ = W.synth_wal(2 << 20, 16, 600, seed=900 + 10 * block + seed,
                                 rewind_per_mille=rng.choice([0, 10]))
            assert_parity(ctx, _mutate(rng, bytes(buf)), 1, check_chain=False)
    finally:
        ctx.set_options()


def test_vh_rewinds_and_auto(ctx):
    """index rewinds (the rewind-mode pass), and the automatic choice: the
    second call on a ctx after a record-dense ReadAll takes the 128-B
    prefixes"""
    li = []
    buf, _ = W.synth_wal(16 << 20, 32, 900, seed=71, rewind_per_mille=15, last_index=li)
    b = bytes(buf)
    o = O.readall_digest(b, 1)
    assert o["status"] == O.OK and o["n_ents"] == li[0]
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        for _ in range(3):   # auto: dense after the first call
            _assert_result(ctx, _readall(ctx, d, len(b), 1, memoryview(b)), o, b)
    finally:
        d.free()
    for vh in (True, False):
        _assert_result(ctx, _dev_readall(ctx, b, 1, vh), o, b)


def test_vh_deferred_range(ctx):
    """a range of a WAL split inside a file, frame 0's check deferred: the
    result and the range info (from the frame pass's reductions) agree with
    the 256-B prefixes and the general path"""
    buf, _ = W.synth_wal(6 << 20, 48, 1200, seed=72)
    b = bytes(buf)
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        start, ri = W.range_probe(d, len(b), 2 << 20, 1 << 20)
    finally:
        d.free()
    assert start > 0 and ri > 1
    part = b[start:]
    d = ctx.alloc(len(part) + 64)
    got = []
    try:
        d.upload(part)
        for general, vh in ((False, True), (False, False), (True, None)):
            ctx.set_options(general_path=general, vh=vh)
            try:
                g = W.readall_range_device(d, len(part), ri, defer_first=True)
                got.append(((g.status, g.n_records, g.last_crc, g.enti), W.range_info(ctx, stream=part)))
            finally:
                ctx.set_options()
    finally:
        d.free()
    assert got[0] == got[1] == got[2]
    assert got[0][0][0] == O.OK


def test_vh_options_validated(ctx):
    with pytest.raises(Exception):
        W.check(L.lib.ewal_ctx_set_options(ctx.handle, L.OPT_VH_ON | L.OPT_VH_OFF))
    ctx.set_options()


def _batch_vs_oracle(ctx, shards, ris, vh):
    ctx.set_options(vh=vh)
    try:
        res = W.readall_batch_bytes(shards, ris, ctx)
    finally:
        ctx.set_options()
    for s, (b, ri, g) in enumerate(zip(shards, ris, res)):
        o = O.readall(b, ri)
        assert g.status == o["status"], (vh, s, g.status, o["status"])
        if o["status"] == O.OK:
            assert (g.n_records, g.last_crc, g.enti, g.metadata) == \
                (o["n_records"], o["last_crc"], o["enti"], o["metadata"]), (vh, s)
            assert [(x.Index, x.Term, x.Data) for x in g.ents] == \
                   [(x["index"], x["term"], x["data"]) for x in o["ents"]], (vh, s)
        elif o["status"] != O.ERR_INDEX_NOT_FOUND:
            assert (g.fail_record, g.fail_offset) == (o["fail_record"], o["fail_offset"]), (vh, s)
    return res


@pytest.mark.parametrize("seed", range(3))
def test_vh_batches_shapes_corrupt_torn_rewinds(ctx, seed):
    """Round 6: the batch frame pass with the 128-B prefixes (k_frames<true,
    TSH, true>; the batch's stream pass stores vh[]) -- record-dense shards of
    several shapes, a corrupt record, a torn tail and a shard after leader
    changes in one batch, with the option on, off and automatic (the second
    automatic call takes it: the first batch was record-dense), every shard
    against the oracle's ReadAll alone."""
    rng = random.Random(9100 + seed)
    shards, ris = [], []
    for i in range(6):
        lo, hi = rng.choice([(16, 300), (64, 1200), (128, 4096), (1, 200)])
        buf, n = W.synth_wal(rng.choice([1, 2, 3]) << 20, lo, hi, seed=300 + 10 * seed + i,
                             corrupt_record=rng.randrange(1, 500) if i == 2 else -1,
                             rewind_per_mille=20 if i == 4 else 0)
        b = bytes(buf)
        if i == 3:
            b = b[:-rng.randrange(1, 200)]   # a torn last frame
        shards.append(b)
        ris.append(1)
    for vh in (True, False, None, None):
        _batch_vs_oracle(ctx, shards, ris, vh)
