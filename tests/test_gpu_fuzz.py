"""GPU parity under mutation: many small WALs, each damaged in one or more of
the ways a disk, a crash or a buggy writer can -- bit flips, torn tails,
inserted / deleted bytes (the frames no longer chain: the general path's
pointer jumping and walker), frames duplicated / dropped / swapped (index
rewinds, gaps, crc seams out of order), trailing garbage -- checked against
the oracle (wal.ReadAll: status, failing frame and offset, ents, state,
metadata, lastCRC), one WAL at a time and as one batch (each shard's
verdict must be its own ReadAll's)."""
import random
import struct

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from test_gpu_parity import assert_parity, build_wal

pytestmark = pytest.mark.gpu


def _frames(buf):
    offs, p = [], 0
    while p + 8 <= len(buf):
        n = struct.unpack_from("<q", buf, p)[0]
        if n < 0 or p + 8 + n > len(buf):
            break
        offs.append((p, 8 + n))
        p += 8 + n
    return offs


def _mutate(rng, w):
    w = bytearray(w)
    for _ in range(rng.choice([1, 1, 1, 2, 3])):
        fr = _frames(bytes(w))
        k = rng.randrange(9)
        if k == 0 and w:                       # bit flips
            for _ in range(rng.randrange(1, 4)):
                p = rng.randrange(len(w))
                w[p] ^= 1 << rng.randrange(8)
        elif k == 1 and w:                     # torn tail
            del w[rng.randrange(len(w)):]
        elif k == 2:                           # inserted bytes
            p = rng.randrange(len(w) + 1)
            w[p:p] = bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 9)))
        elif k == 3 and len(w) > 1:            # deleted bytes
            p = rng.randrange(len(w) - 1)
            del w[p:p + rng.randrange(1, 9)]
        elif k == 4 and len(fr) > 3:           # a frame duplicated (an index rewind by one)
            p, n = fr[rng.randrange(2, len(fr))]
            w[p + n:p + n] = w[p:p + n]
        elif k == 5 and len(fr) > 3:           # a frame dropped (crc mismatch / index gap)
            p, n = fr[rng.randrange(2, len(fr))]
            del w[p:p + n]
        elif k == 6 and len(fr) > 4:           # two neighbouring frames swapped
            i = rng.randrange(2, len(fr) - 1)
            (p, n), (q, m) = fr[i], fr[i + 1]
            w[p:q + m] = w[q:q + m] + w[p:p + n]
        elif k == 7:                           # trailing garbage / a bare length prefix
            w += (struct.pack("<q", rng.randrange(-5, 3000)) if rng.random() < 0.5
                  else bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 24))))
        elif k == 8 and len(fr) > 2:           # a length prefix rewritten
            p, n = fr[rng.randrange(len(fr))]
            struct.pack_into("<q", w, p, max(0, n - 8 + rng.choice([-3, -1, 1, 2, 64])))
    return bytes(w)


@pytest.mark.parametrize("block", range(10))
def test_mutated_wals(ctx, block):
    rng = random.Random(7000 + block)
    seen = set()
    for _ in range(60):
        w = build_wal(rng, rng.randrange(3, 90), rng.choice([40, 600, 5000]), cuts=rng.randrange(0, 3),
                      big_terms=rng.random() < 0.3)
        m = _mutate(rng, w)
        ri = rng.choice([0, 0, 1, 3, 40])
        o, g = assert_parity(ctx, m, ri)
        assert g["status"] != L.UNSUPPORTED_ENCODING
        seen.add(o["status"])
    assert len(seen) >= 3   # the mutations reach several verdicts


@pytest.mark.parametrize("vh", [None, True])
@pytest.mark.parametrize("block", range(5))
def test_mutated_batches(ctx, block, vh):
    ctx.set_options(vh=vh)
    try:
        _mutated_batches(ctx, block)
    finally:
        ctx.set_options()


def _mutated_batches(ctx, block):
    rng = random.Random(9100 + block)
    for _ in range(6):
        shards, ris = [], []
        for _ in range(rng.randrange(2, 12)):
            w = build_wal(rng, rng.randrange(3, 60), rng.choice([40, 600, 3000]), cuts=rng.randrange(0, 2),
                          big_terms=False)
            shards.append(_mutate(rng, w) if rng.random() < 0.5 else w)
            ris.append(rng.choice([0, 1, 5]))
        res = W.readall_batch_bytes(shards, ris, ctx)
        for s, ri, r in zip(shards, ris, res):
            o = O.readall(s, ri)
            assert r.status == o["status"], (r.status, o["status"])
            if o["status"] == O.OK:
                assert r.metadata == o["metadata"]
                assert [(x.Index, x.Term, x.Data) for x in r.ents] == \
                       [(x["index"], x["term"], x["data"]) for x in o["ents"]]
            elif o["status"] != O.ERR_INDEX_NOT_FOUND:
                assert (r.fail_record, r.fail_offset) == (o["fail_record"], o["fail_offset"])


@pytest.mark.parametrize("seed", range(12))
def test_mutated_large_wals(ctx, seed):
    # multi-MiB WALs (thousands of 64-frame tiles, rewinds for some seeds): the
    # damage lands far from byte 0, across tile seams, in the fused pass and in
    # the general path's pointer jumping
    rng = random.Random(11000 + seed)
    size = rng.choice([1, 3, 8]) << 20
    buf, _ = W.synth_wal(size, rng.choice([16, 64]), rng.choice([512, 4096]), seed=seed,
                         rewind_per_mille=rng.choice([0, 0, 10]))
    m = _mutate(rng, bytes(buf))
    o, g = assert_parity(ctx, m, rng.choice([1, 1, 100]), check_chain=seed % 3 == 0)   # its entries start at Index 1
    assert g["status"] != L.UNSUPPORTED_ENCODING


def _large_case(seed):
    """a multi-MiB WAL whose entries may span whole frame-pass tiles (up to
    150 KiB), leader changes for some seeds, mutated for 60 % of the seeds"""
    rng = random.Random(13000 + seed)
    size = rng.choice([2, 6, 12]) << 20
    hi = rng.choice([4096, 65536, 150 << 10])
    buf, _ = W.synth_wal(size, rng.choice([16, 64, 2048]), hi, seed=100 + seed,
                         rewind_per_mille=rng.choice([0, 10, 30]))
    b = bytes(buf)
    return (_mutate(rng, b) if rng.random() < 0.6 else b), rng.choice([1, 1, 50])


@pytest.mark.parametrize("seed", range(8))
def test_mutated_wals_with_tile_spanning_entries(ctx, seed):
    m, ri = _large_case(seed)
    o, g = assert_parity(ctx, m, ri, check_chain=seed % 4 == 0)
    assert g["status"] != L.UNSUPPORTED_ENCODING


def _large_batch_case(seed):
    """3-8 multi-MiB shards of the large case's kinds (tile-spanning entries,
    leader changes, mutations) side by side in one batch"""
    rng = random.Random(17000 + seed)
    shards, ris = [], []
    for i in range(rng.randrange(3, 9)):
        buf, _ = W.synth_wal(rng.choice([1, 3, 5]) << 20, rng.choice([16, 64, 2048]),
                             rng.choice([4096, 65536, 150 << 10]), seed=200 + 16 * seed + i,
                             rewind_per_mille=rng.choice([0, 10, 30]))
        b = bytes(buf)
        shards.append(_mutate(rng, b) if rng.random() < 0.4 else b)
        ris.append(rng.choice([1, 1, 50]))
    return shards, ris


def check_batch(ctx, shards, ris):
    res = W.readall_batch_bytes(shards, ris, ctx)
    for s, ri, r in zip(shards, ris, res):
        o = O.readall(s, ri)
        assert r.status == o["status"], (r.status, o["status"])
        if o["status"] == O.OK:
            assert (r.n_records, r.last_crc, r.enti, r.metadata) == \
                (o["n_records"], o["last_crc"], o["enti"], o["metadata"])
            assert [(x.Index, x.Term, x.Data) for x in r.ents] == \
                   [(x["index"], x["term"], x["data"]) for x in o["ents"]]
        elif o["status"] != O.ERR_INDEX_NOT_FOUND:
            assert (r.fail_record, r.fail_offset) == (o["fail_record"], o["fail_offset"])
    return res


@pytest.mark.parametrize("vh", [None, True])
@pytest.mark.parametrize("seed", range(4))
def test_mutated_batches_with_tile_spanning_entries(ctx, seed, vh):
    ctx.set_options(vh=vh)
    try:
        check_batch(ctx, *_large_batch_case(seed))
    finally:
        ctx.set_options()
