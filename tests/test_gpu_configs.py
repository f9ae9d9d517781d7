"""GPU parity at BASELINE.json's config sizes.

* configs[0]: a WAL of 1M x 256 B entries (wal.Save's layout: crc, metadata,
  HardState, entries; ~286 MB) -- the whole ReadAll result against the
  oracle's: status, frames, lastCRC, enti, metadata, HardState, the ents (a
  digest over every entry's fields and Data) and all 1M chained CRCs.
* configs[2]: 512 per-raft-group WAL shards x 64 MiB in ONE batched ReadAll
  (32 GiB, ~29 M frames: more than 2^24 frames, the segmented check spans
  many 1 GiB tile groups): every clean shard OK with its exact frame count,
  the corrupt shard's walpb.ErrCRCMismatch at its exact frame, no shard on
  the one-by-one fallback; the faithful oracle's full result (ents digest
  included) on a sample of shards, the optimised C restatement's full result
  (every entry descriptor) on all the others.
* configs[3]: snapshot files of 1-256 MiB (log-uniform) in one
  esnap_verify_packed call against or_loadsnap, corrupt files included.

References: wal/wal.go:164-216, wal/decoder.go:28-47, snap/snapshotter.go:76-111.
"""
import ctypes as C
import math
import random

import numpy as np
import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W
from etcd_amd import snap as S

pytestmark = pytest.mark.gpu


def _device_ents_digest(ctx, buf, n, shard=None):
    arr = (L.EntryDesc * max(n, 1))()
    k = L.lib.ewal_copy_entries(ctx.handle, arr, n) if shard is None else \
        L.lib.ewal_batch_copy_entries(ctx.handle, shard, arr, n)
    assert k == n
    return O.ent_views_digest(buf, arr, n)


def _assert_result(ctx, g, o, buf, shard=None):
    assert (g.status, g.fail_record, g.fail_offset) == (o["status"], o["fail_record"], o["fail_offset"])
    if o["status"] != O.OK:
        return
    assert (g.n_records, g.last_crc, g.enti) == (o["n_records"], o["last_crc"], o["enti"])
    assert g.metadata == o["metadata"]
    assert (g.state.Term, g.state.Vote, g.state.Commit) == o["state"]
    assert g.n_ents == o["n_ents"]
    assert _device_ents_digest(ctx, buf, g.n_ents, shard) == o["ents_digest"]


def _readall(ctx, dbuf, nb, ri, host):
    r = L.Result()
    rc = L.lib.ewal_readall_device(ctx.handle, dbuf.ptr, nb, ri, C.byref(r))
    assert rc >= 0, rc
    res = W._collect(ctx, r, host, with_ents=False)
    res.n_ents = r.n_ents
    return res


def test_configs0_1m_x_256b(ctx):
    buf, n = W.synth_wal(285_000_000, 256, 256, seed=1)
    b = bytes(buf)
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        g = _readall(ctx, d, len(b), 1, memoryview(b))
        o = O.readall_digest(b, 1)
        assert o["status"] == O.OK and o["n_ents"] > 990_000
        _assert_result(ctx, g, o, b)
        # every chained CRC and frame offset
        crcs, offs = O.chain_crcs(b, cap=n + 16)
        recs = (L.RecordDesc * n)()
        assert L.lib.ewal_copy_records(ctx.handle, recs, n) == n
        ra = np.frombuffer(recs, dtype=np.dtype([("offset", "<u8"), ("data_off", "<u8"), ("data_len", "<u8"),
                                                 ("type", "<i8"), ("crc", "<u4"), ("chained_crc", "<u4")]))
        assert np.array_equal(ra["chained_crc"], np.array(crcs, dtype=np.uint32))
        assert np.array_equal(ra["offset"], np.array(offs, dtype=np.uint64))
        # one corrupt record in the middle
        k = n // 2
        p = int(ra["data_off"][k]) + int(ra["data_len"][k]) // 2
        bad = bytearray(b)
        bad[p] ^= 0x01
        d.upload(bytes(bad[p:p + 1]), p)
        g = _readall(ctx, d, len(b), 1, memoryview(bad))
        o = O.readall_digest(bytes(bad), 1)
        assert o["status"] == O.ERR_RECORD_CRC and o["fail_record"] == k
        _assert_result(ctx, g, o, bytes(bad))
    finally:
        d.free()


def test_configs1_full_size_against_oracle(ctx):
    """configs[1] at its full size (8 GiB, mixed 64 B - 64 KiB entries, the
    bench's WAL): the whole ReadAll result against the oracle's over the same
    bytes -- clean: status, frames, lastCRC, enti, metadata, HardState and the
    ents digest against the faithful restatement (or_readall), and every
    entry descriptor (term, index, Data offset + length, type, nil flag)
    against the optimised restatement (orf_readall, pinned to or_readall by
    tests/test_cpu_baseline.py); with one flipped payload byte at frame
    k = 0.73 N: status, fail_record and fail_offset against both.
    Reference: wal/wal.go:164-216, wal/decoder.go:28-47."""
    buf, n = W.synth_wal(8 << 30, 64, 65536, seed=2)
    nb = len(buf)
    d = ctx.alloc(nb + 64)
    try:
        d.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
        hb = bytes(buf)
        o = O.readall_digest(hb, 1)
        assert o["status"] == O.OK and o["n_records"] == n
        g = _readall(ctx, d, nb, 1, buf)
        _assert_result(ctx, g, o, hb)
        # every entry descriptor against the optimised restatement
        raw = (C.c_char * nb).from_buffer(buf)
        fr = O.FastResult()
        st = O.lib.orf_readall(C.c_void_p(C.addressof(raw)), nb, 1, 16, C.byref(fr))
        try:
            assert st != O.IRREGULAR
            assert (fr.status, fr.n_records, fr.last_crc, fr.enti, fr.n_ents) == \
                (g.status, g.n_records, g.last_crc, g.enti, g.n_ents)
            ne = int(fr.n_ents)
            got = (L.EntryDesc * max(ne, 1))()
            assert L.lib.ewal_copy_entries(ctx.handle, got, ne) == ne
            want = np.frombuffer(C.string_at(fr.ents, ne * _ENT_DT.itemsize), dtype=_ENT_DT)
            assert np.array_equal(np.frombuffer(got, dtype=_ENT_DT)[:ne], want)
        finally:
            O.lib.orf_result_free(C.byref(fr))
        del raw
        # one corrupt record at k = 0.73 N (the bench's), device and host alike
        k = int(0.73 * n)
        rec = W.records(ctx, n)[k]
        p = rec["data_off"] + rec["data_len"] // 2
        b = bytearray(d.download(1, p))
        b[0] ^= 0x5A
        d.upload(bytes(b), p)
        buf[p] ^= 0x5A
        del hb
        hb = bytes(buf)
        o2 = O.readall_digest(hb, 1)
        assert o2["status"] == O.ERR_RECORD_CRC and o2["fail_record"] == k
        g2 = _readall(ctx, d, nb, 1, buf)
        _assert_result(ctx, g2, o2, hb)
        assert g2.fail_offset == rec["offset"]
        f2 = O.fast_readall_status(C.addressof((C.c_char * nb).from_buffer(buf)), nb, 1, 16)
        assert f2[0] == O.ERR_RECORD_CRC and f2[2] == k
    finally:
        d.free()


def test_configs2_512_shards_x_64mib(ctx):
    nsh, bad_shard, bad_rec = 512, 2749 % 512, 1000
    blob, lens, nrec = W.synth_shards(list(range(nsh)), 64 << 20, 128, 4096, corrupt={bad_shard: bad_rec})
    assert sum(nrec) > (1 << 24)
    d = ctx.alloc(len(blob) + 64)
    try:
        d.upload_ptr(C.addressof((C.c_char * len(blob)).from_buffer(blob)), len(blob))
        out = (L.Result * nsh)()
        rc = L.lib.ewal_readall_batch_device(ctx.handle, d.ptr, nsh, (C.c_uint64 * nsh)(*lens),
                                             (C.c_uint64 * nsh)(*([1] * nsh)), out)
        assert rc == 0, rc
        for s in range(nsh):
            r = out[s]
            assert not (r.flags & L.FLAG_SHARD_FALLBACK), s
            if s == bad_shard:
                assert (r.status, r.fail_record) == (L.ERR_RECORD_CRC, bad_rec), (s, r.status, r.fail_record)
            else:
                assert (r.status, r.n_records) == (L.OK, nrec[s]), (s, r.status, r.n_records, nrec[s])
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        rng = random.Random(2)
        sample = sorted({0, 1, bad_shard, nsh - 1} | set(rng.sample(range(nsh), 4)))
        for s in sample:
            sb = bytes(blob[offs[s]:offs[s + 1]])
            o = O.readall_digest(sb, 1)
            g = W._collect(ctx, out[s], memoryview(sb), with_ents=False, shard=s)
            g.n_ents = out[s].n_ents
            _assert_result(ctx, g, o, sb, shard=s)
        # every other shard's whole result against the optimised C restatement
        # (orf_readall, pinned to the faithful or_readall by
        # tests/test_cpu_baseline.py): the verdict fields and every entry
        # descriptor (Data as offset + length into the shard, so equal views
        # mean equal bytes)
        _all_shards_vs_fast_oracle(ctx, blob, offs, lens, out, skip=set(sample))
    finally:
        d.free()


_ENT_DT = np.dtype([("term", "<u8"), ("index", "<u8"), ("data_off", "<u8"), ("data_len", "<u8"), ("type", "<i4"),
                    ("data_nil", "<i4")])


def _all_shards_vs_fast_oracle(ctx, blob, offs, lens, out, skip):
    raw = (C.c_char * len(blob)).from_buffer(blob)
    base = C.addressof(raw)
    checked = 0
    for s in range(len(lens)):
        if s in skip:
            continue
        fr = O.FastResult()
        st = O.lib.orf_readall(C.c_void_p(base + int(offs[s])), int(lens[s]), 1, 8, C.byref(fr))
        try:
            assert st != O.IRREGULAR, s
            r = out[s]
            assert (r.status, r.fail_record, r.n_records, r.last_crc, r.enti, r.n_ents) == \
                (fr.status, fr.fail_record, fr.n_records, fr.last_crc, fr.enti, fr.n_ents), s
            assert (r.metadata_off, r.metadata_len) == (fr.metadata_off, fr.metadata_len), s
            assert (r.has_state, r.state_term, r.state_vote, r.state_commit) == \
                (fr.has_state, fr.state_term, fr.state_vote, fr.state_commit), s
            n = int(fr.n_ents)
            got = (L.EntryDesc * max(n, 1))()
            assert L.lib.ewal_batch_copy_entries(ctx.handle, s, got, n) == n
            want = np.frombuffer(C.string_at(fr.ents, n * _ENT_DT.itemsize) if n else b"", dtype=_ENT_DT)
            assert np.array_equal(np.frombuffer(got, dtype=_ENT_DT)[:n], want), s
            checked += 1
        finally:
            O.lib.orf_result_free(C.byref(fr))
    del raw
    assert checked == len(lens) - len(skip)


def test_configs3_snapshots_1_to_256mib(ctx):
    rng, crng = random.Random(4), random.Random(5)
    pool = np.random.default_rng(4).integers(0, 256, size=(256 << 20) + 4096, dtype=np.uint8).tobytes()
    sizes = [int(math.exp(rng.uniform(math.log(1 << 20), math.log(64 << 20)))) for _ in range(14)] + [(256 << 20) - 64]
    files, bad = [], []
    for i, n in enumerate(sizes):
        st = rng.randrange(0, len(pool) - n)
        f = bytearray(S.snap_file(S.snapshot_marshal(pool[st:st + n], (1, 2, 3), i + 1, 1)))
        if i in (3, 9) or crng.random() < 0.05:
            f[crng.randrange(len(f) // 4, len(f))] ^= 0x10
            bad.append(i)
        files.append(bytes(f))
    offs, pos = [], 0
    for f in files:
        offs.append(pos)
        pos += len(f) + 16            # files need not be packed back to back
    packed = bytearray(pos)
    for o_, f in zip(offs, files):
        packed[o_:o_ + len(f)] = f
    d = ctx.alloc(len(packed) + 64)
    try:
        d.upload_ptr(C.addressof((C.c_char * len(packed)).from_buffer(packed)), len(packed))
        st, sc, cc = S.verify_packed(d, len(packed), offs, [len(f) for f in files])
        for i, f in enumerate(files):
            o = O.loadsnap(f)
            assert st[i] == o["status"], (i, st[i], o["status"])
            assert (sc[i], cc[i]) == (o["stored_crc"], o["computed_crc"]), i
            if o["status"] == O.OK:
                s = L.SnapshotDesc()
                assert L.lib.esnap_copy_snapshot(ctx.handle, i, C.byref(s)) == 0
                assert (s.index, s.term, list(s.nodes[:s.n_nodes])) == (i + 1, 1, [1, 2, 3])
                assert packed[s.data_off:s.data_off + s.data_len] == o["snap"]["data"]
        assert [i for i in range(len(files)) if st[i] != L.OK] == bad
    finally:
        d.free()


def test_configs3_ten_k_distribution_sample(ctx):
    """192 files drawn from configs[3]'s 10k-file size distribution
    (log-uniform 1-256 MiB, ~9 GiB, ~2 % corrupt: a flipped byte in the body,
    the stored CRC or the envelope) in one esnap_verify_packed call: every
    file's verdict and computed CRC against the optimised C restatement
    (orf_snap_verify_batch, pinned to or_loadsnap by
    tests/test_cpu_baseline.py), the faithful or_loadsnap on 12 of them."""
    rng, crng = random.Random(14), random.Random(15)
    pool = np.random.default_rng(14).integers(0, 256, size=(256 << 20) + 4096, dtype=np.uint8).tobytes()
    sizes = [int(math.exp(rng.uniform(math.log(1 << 20), math.log(256 << 20)))) for _ in range(192)]
    offs, lens, pos = [], [], 0
    for n in sizes:
        offs.append(pos)
        lens.append(n + 64)           # upper bound of the envelope; trimmed below
        pos += (n + 64 + 15) & ~15
    packed = bytearray(pos)
    bad = []
    for i, n in enumerate(sizes):
        st = rng.randrange(0, len(pool) - n)
        f = bytearray(S.snap_file(S.snapshot_marshal(pool[st:st + n], (1, 2, 3), i + 1, 1)))
        if i in (5, 77, 150) or crng.random() < 0.02:
            f[crng.choice([1, 3, len(f) // 2, len(f) - 1])] ^= 0x10   # stored CRC, envelope length, body
            bad.append(i)
        lens[i] = len(f)
        packed[offs[i]:offs[i] + len(f)] = f
    del pool
    d = ctx.alloc(len(packed) + 64)
    try:
        raw = (C.c_char * len(packed)).from_buffer(packed)
        d.upload_ptr(C.addressof(raw), len(packed))
        st, sc, cc = S.verify_packed(d, len(packed), offs, lens)
        fst, fcc = O.fast_snap_verify_batch(C.addressof(raw), offs, lens, 8)
        assert st == fst
        assert [cc[i] for i in range(len(sizes)) if st[i] == L.OK] == [fcc[i] for i in range(len(sizes)) if fst[i] == O.OK]
        assert all(st[i] != L.OK for i in bad)
        assert sum(1 for x in st if x != L.OK) == len(bad)
        for i in sorted(set(bad[:6]) | set(random.Random(16).sample(range(len(sizes)), 6))):
            o = O.loadsnap(bytes(packed[offs[i]:offs[i] + lens[i]]))
            assert st[i] == o["status"], (i, st[i], o["status"])
            if o["status"] in (O.OK, O.ERR_SNAP_CRC):
                assert (sc[i], cc[i]) == (o["stored_crc"], o["computed_crc"]), i
        del raw
    finally:
        d.free()


@pytest.mark.gpu
def test_configs4_1m_groups_against_oracle(ctx):
    """configs[4] at its full size: maybeCommit (raft/raft.go:248-258 +
    raft/log.go:148-154) over 1M raft groups x 5/7 voters with a 16-entry
    log-term window (bench.py's generator, seed 6, plus groups whose quorum
    index falls outside the window: no change / Go's bounds panic) -- every
    committed index, changed flag and status against or_maybe_commit_batch."""
    import numpy as np
    import torch
    G = 1 << 20
    rng = np.random.default_rng(6)
    nv = np.where(rng.random(G) < 0.5, 5, 7).astype(np.uint8)
    committed0 = rng.integers(0, 1 << 20, size=G, dtype=np.uint64)
    match = (committed0[None, :] + rng.integers(0, 24, size=(7, G), dtype=np.uint64) - np.uint64(4)).astype(np.uint64)
    term = rng.integers(1, 4, size=G, dtype=np.uint64)
    log_offset = committed0 + np.uint64(1) - rng.integers(0, 3, size=G, dtype=np.uint64)
    # a slice of groups whose log window ends early (at() past the log: the bounds panic) or has no voters
    short = rng.random(G) < 0.01
    lens = np.where(short, rng.integers(0, 4, size=G), 16).astype(np.uint64)
    log_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    log_terms = rng.integers(1, 4, size=int(lens.sum()), dtype=np.uint64)
    nv[rng.random(G) < 0.001] = 0
    dev = torch.device("cuda", 0)
    T = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)   # noqa: E731
    d = dict(m=T(match.reshape(-1)), n=T(nv), t=T(term), c=T(committed0.copy()), o=T(log_offset), p=T(log_ptr),
             lt=T(log_terms))
    ch = torch.zeros(G, dtype=torch.uint8, device=dev)
    st = torch.zeros(G, dtype=torch.uint8, device=dev)
    P = lambda t: C.c_void_p(t.data_ptr())   # noqa: E731
    assert L.lib.ecommit_batch_device(ctx.handle, G, P(d["m"]), P(d["n"]), P(d["t"]), P(d["c"]), P(d["o"]), P(d["p"]),
                                      P(d["lt"]), P(ch), P(st), None) == 0
    c = committed0.copy()
    chc, stc = np.zeros(G, np.uint8), np.zeros(G, np.uint8)
    O.maybe_commit_batch(G, match.reshape(-1).copy(), nv, term, c, log_offset, log_ptr, log_terms, chc, stc)
    got_c = d["c"].cpu().numpy().view(np.uint64)
    assert (stc != 0).sum() > 0 and chc.sum() > G // 4
    np.testing.assert_array_equal(st.cpu().numpy(), stc)
    np.testing.assert_array_equal(ch.cpu().numpy(), chc)
    ok = stc == 0
    np.testing.assert_array_equal(got_c[ok], c[ok])
    # the same groups as 128-B records (ecommit_batch_rec_device): the quorum
    # index's term from the record's tail window, else the log_terms gather
    from etcd_amd import raftcommit as RC
    rec = T(RC.pack_groups(match, nv, committed0, term, log_offset, log_ptr, log_terms).reshape(-1))
    co = torch.zeros(G, dtype=torch.int64, device=dev)
    ch.zero_()
    st.zero_()
    assert L.lib.ecommit_batch_rec_device(ctx.handle, G, P(rec), P(d["p"]), P(d["lt"]), P(co), P(ch), P(st), None) == 0
    np.testing.assert_array_equal(st.cpu().numpy(), stc)
    np.testing.assert_array_equal(ch.cpu().numpy(), chc)
    np.testing.assert_array_equal(co.cpu().numpy().view(np.uint64)[ok], c[ok])
    # without the log arrays: only groups whose quorum term lies before the window lose their verdict
    assert L.lib.ecommit_batch_rec_device(ctx.handle, G, P(rec), None, None, P(co), P(ch), P(st), None) == 0
    st2 = st.cpu().numpy()
    moved = st2 != stc
    assert (st2[moved] == L.UNSUPPORTED_ENCODING).all() and moved.sum() < G // 10
    np.testing.assert_array_equal(co.cpu().numpy().view(np.uint64)[ok & ~moved], c[ok & ~moved])


@pytest.mark.gpu
def test_configs1_shaped_with_leader_changes(ctx):
    """A configs[1]-shaped WAL (64 B - 64 KiB entries) where 1 % of the entries
    open a new leader's term that rewrites the last 1..8 indexes (wal/wal.go:173
    truncate-and-overwrite): every ents Index / Term / Data view against the
    oracle's ReadAll, single WAL and as one shard of a batch beside clean ones.
    Both on the frame pass (its rewind mode), no general path and no shard
    replayed alone."""
    li = []
    buf, n = W.synth_wal(96 << 20, 64, 65536, seed=12, rewind_per_mille=10, last_index=li)
    b = bytes(buf)
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        g = _readall(ctx, d, len(b), 1, memoryview(b))
        o = O.readall_digest(b, 1)
        assert o["status"] == O.OK and o["n_ents"] == li[0]
        _assert_result(ctx, g, o, b)
        assert g.flags & L.FLAG_FAST_PATH
    finally:
        d.free()
    clean = [bytes(W.synth_wal(8 << 20, 64, 16384, seed=30 + i)[0]) for i in range(3)]
    small = bytes(W.synth_wal(16 << 20, 64, 16384, seed=13, rewind_per_mille=10)[0])
    shards = [clean[0], small, clean[1], clean[2]]
    res = W.readall_batch_bytes(shards, [1] * 4, ctx, with_ents=True)
    for s, (sb, r) in enumerate(zip(shards, res)):
        o = O.readall(sb, 1)
        assert r.status == o["status"] == O.OK and (r.n_records, r.last_crc, r.enti) == \
            (o["n_records"], o["last_crc"], o["enti"])
        assert [(e.Index, e.Term, e.Data) for e in r.ents] == [(e["index"], e["term"], e["data"]) for e in o["ents"]]
        assert not (r.flags & L.FLAG_SHARD_FALLBACK)


@pytest.mark.gpu
@pytest.mark.parametrize("rewinds", [0, 20])
def test_tiles_without_frames_after_dense_call(ctx, rewinds):
    """Tiles that hold no frame start (entries of 64-160 KiB span whole tiles)
    after a record-dense call on the same ctx left every tile's op fields set:
    the seam pass's gap rule must skip the empty tiles by their frame count,
    not by op fields the frame pass writes only for tiles with frames
    (wal/wal.go:170-176; round 5: stale fields read as the predecessor op gave
    a false index-gap panic)."""
    dense = bytes(W.synth_wal(24 << 20, 32, 600, seed=77)[0])
    li = []
    big = bytes(W.synth_wal(24 << 20, 64 << 10, 160 << 10, seed=78, rewind_per_mille=rewinds, last_index=li)[0])
    for b, check_n in ((dense, False), (big, True), (dense, False), (big, True)):
        d = ctx.alloc(len(b) + 64)
        try:
            d.upload(b)
            g = _readall(ctx, d, len(b), 1, memoryview(b))
        finally:
            d.free()
        o = O.readall_digest(b, 1)
        assert o["status"] == O.OK
        if check_n:
            assert o["n_ents"] == li[0]
        _assert_result(ctx, g, o, b)


@pytest.mark.gpu
def test_ctx_reuse_across_shapes(ctx):
    """One ctx through a mixed sequence of single and batched ReadAlls whose
    shapes differ call to call (record-dense, entries spanning whole tiles,
    leader changes, corrupt and torn WALs, a one-frame WAL): every per-call
    device buffer a call reads must be one it wrote, so each result equals
    the oracle's whatever the previous call left behind (wal/wal.go:164-216)."""
    def shape(kind, seed):
        if kind == "dense":
            return bytes(W.synth_wal(6 << 20, 16, 400, seed=seed)[0])
        if kind == "big":
            return bytes(W.synth_wal(12 << 20, 64 << 10, 150 << 10, seed=seed, rewind_per_mille=30)[0])
        if kind == "c1":
            return bytes(W.synth_wal(20 << 20, 64, 65536, seed=seed, rewind_per_mille=10)[0])
        if kind == "corrupt":
            return bytes(W.synth_wal(5 << 20, 32, 3000, seed=seed, corrupt_record=1500)[0])
        if kind == "torn":
            b = bytes(W.synth_wal(4 << 20, 32, 5000, seed=seed)[0])
            return b[:-(seed % 200 + 1)]
        return bytes(W.synth_wal(1, 8, 8, seed=seed)[0])   # "one": the smallest WAL the generator writes
    rng = random.Random(4242)
    kinds = ["dense", "big", "c1", "corrupt", "torn", "one"]
    for step in range(14):
        if step % 3 == 2:   # a batch of three different shapes
            ks = rng.sample(kinds, 3)
            shards = [shape(k, 900 + 10 * step + i) for i, k in enumerate(ks)]
            res = W.readall_batch_bytes(shards, [1] * 3, ctx, with_ents=True)
            for sb, r, k in zip(shards, res, ks):
                o = O.readall(sb, 1)
                assert (r.status, r.fail_record, r.fail_offset) == (o["status"], o["fail_record"], o["fail_offset"]), k
                if o["status"] == O.OK:
                    assert (r.n_records, r.last_crc, r.enti) == (o["n_records"], o["last_crc"], o["enti"]), k
                    assert [(e.Index, e.Term, e.Data) for e in r.ents] == \
                        [(e["index"], e["term"], e["data"]) for e in o["ents"]], k
            continue
        k = kinds[rng.randrange(len(kinds))]
        b = shape(k, 700 + step)
        d = ctx.alloc(len(b) + 64)
        try:
            d.upload(b)
            g = _readall(ctx, d, len(b), 1, memoryview(b))
        finally:
            d.free()
        _assert_result(ctx, g, O.readall_digest(b, 1), b)


@pytest.mark.gpu
def test_records_and_range_info_after_rewinding_readall_keep_ents(ctx):
    """ewal_copy_records / ewal_copy_range_info after a frame-pass ReadAll
    that met index rewinds rebuild the per-frame descriptors on demand; the
    call's ents (rewinds applied, wal/wal.go:173) must be unchanged by that
    (round 5: the rebuild's k_check overwrote them with the ops in order,
    found by splitting such a WAL over two ctxs)."""
    li = []
    b = bytes(W.synth_wal(8 << 20, 64, 4096, seed=91, rewind_per_mille=30, last_index=li)[0])
    o = O.readall_digest(b, 1)
    assert o["status"] == O.OK and o["n_ents"] == li[0] < o["n_records"]
    d = ctx.alloc(len(b) + 64)
    try:
        d.upload(b)
        g = _readall(ctx, d, len(b), 1, memoryview(b))
        assert g.flags & L.FLAG_FAST_PATH
        _assert_result(ctx, g, o, b)
        recs = W.records(ctx, g.n_records)
        assert len(recs) == o["n_records"]
        W.range_info(ctx, stream=b)
        _assert_result(ctx, g, o, b)   # the ents again, after both
    finally:
        d.free()
