"""ctx state across calls: the per-frame descriptors of a ReadAll
decided by the fused pass are rebuilt on demand from the ctx's stream-pass
state, so any later compute call that replaces that state must make
ewal_copy_records / ewal_copy_range_info fail (EWAL_E_INVAL) instead of
returning descriptors of the wrong stream."""
import ctypes as C

import pytest

from etcd_amd import wal as W, _lib as L
from oracle import oracle as O


def _wal(ctx, seed=5):
    buf, n = W.synth_wal(1 << 20, 64, 4096, seed=seed)
    d = ctx.alloc(len(buf) + 64)
    d.upload(bytes(buf))
    return bytes(buf), n, d


def _records_fail(ctx, n):
    with pytest.raises(L.EwalError) as e:
        W.records(ctx, n)
    assert e.value.status == L.E_INVAL


@pytest.mark.gpu
def test_records_match_oracle_then_invalidate(ctx):
    buf, n, d = _wal(ctx)
    try:
        r = W.readall_device(d, len(buf), 1)
        assert r.status == L.OK and r.n_records == n
        recs = W.records(ctx, n)
        want, offs = O.chain_crcs(buf)
        assert [x["offset"] for x in recs] == offs[:n]
        assert [x["chained_crc"] for x in recs] == want[:n]
        # a CRC call runs the stream pass again: the descriptors are gone
        out = C.c_uint32()
        L.check(L.lib.ewal_crc32_update_device(ctx.handle, 0, L.CASTAGNOLI, d.ptr, 4096, C.byref(out)))
        assert out.value == O.crc32_update(0, buf[:4096])
        _records_fail(ctx, n)
        with pytest.raises(L.EwalError):
            W.range_info(ctx, stream=buf)
        # a batched ReadAll replaces them too
        W.readall_device(d, len(buf), 1)
        assert len(W.records(ctx, 8)) == 8
        rs = W.readall_batch_device(d, [len(buf)], [1])
        assert rs[0].status == L.OK
        _records_fail(ctx, n)
        # a ReadAll over host bytes stages them; staging new bytes before the
        # descriptors were rebuilt takes their stream away (once rebuilt they
        # hold offsets and CRCs only and stay valid until the next pipeline call)
        g = W.readall_bytes(buf, 1, ctx, with_ents=False)
        assert g.status == L.OK
        p = C.c_void_p()
        L.check(L.lib.ewal_stage_to_device(ctx.handle, b"\0" * 64, 64, C.byref(p)))
        _records_fail(ctx, n)
        # a fresh ReadAll makes them available again
        W.readall_device(d, len(buf), 1)
        assert [x["chained_crc"] for x in W.records(ctx, n)] == want[:n]
    finally:
        d.free()


@pytest.mark.gpu
def test_path_is_set_by_options_not_environment(monkeypatch):
    """the product build reads no environment variable that
    switches the ReadAll path.  A fresh ctx created with the old switches set
    still takes the fused pass (EWAL_FLAG_FAST_PATH); only
    ewal_ctx_set_options(EWAL_OPT_GENERAL_PATH) moves it to the general path,
    with the same verdict and chained CRC."""
    monkeypatch.setenv("EWAL_FUSED", "0")
    monkeypatch.setenv("EWAL_FRAME_WG", "1")
    buf, n = W.synth_wal(2 << 20, 64, 4096, seed=11)
    buf = bytes(buf)
    o = O.readall(buf, 1)
    c = W.Context(0)
    try:
        d = c.alloc(len(buf) + 64)
        d.upload(buf)
        r = W.readall_device(d, len(buf), 1)
        assert r.flags & L.FLAG_FAST_PATH
        assert (r.status, r.n_records, r.last_crc) == (O.OK, o["n_records"], o["last_crc"])
        c.set_options(general_path=True)
        g = W.readall_device(d, len(buf), 1)
        assert not (g.flags & L.FLAG_FAST_PATH)
        assert (g.status, g.n_records, g.last_crc, g.enti) == (r.status, r.n_records, r.last_crc, r.enti)
        c.set_options(general_path=False)
        assert W.readall_device(d, len(buf), 1).flags & L.FLAG_FAST_PATH
        d.free()
    finally:
        c.close()
