"""Host-side mirror of etcd's `wal` package over the MI355X engine.

Names, argument meaning and error behaviour follow the reference
(mzsanford/etcd v0.5.0-alpha):
  OpenAtIndex(dirpath, index)      wal/wal.go:108-159
  WAL.ReadAll() -> (metadata, state, ents)   wal/wal.go:164-216
  Create(dirpath, metadata) / SaveEntry / SaveState / Save / Cut / Sync / Close
                                   wal/wal.go:72-100, 219-292
Errors are raised as exceptions carrying the Go sentinel they stand for
(see ERRORS); Go panics are raised as GoPanic.  All verification runs on
the GPU through libewal.so.
"""
import atexit
import ctypes as C
import weakref
from dataclasses import dataclass, field
from typing import List, Optional

from . import _lib as L
from ._lib import lib, check, EwalError, GoPanic  # noqa: F401

# Go sentinel name for each status (for messages and test readability)
ERRORS = {
    L.ERR_UNEXPECTED_EOF: "io.ErrUnexpectedEOF",
    L.ERR_RECORD_CRC: "walpb.ErrCRCMismatch",
    L.ERR_WAL_CRC: "wal.ErrCRCMismatch",
    L.ERR_METADATA_CONFLICT: "wal.ErrMetadataConflict",
    L.ERR_INDEX_NOT_FOUND: "wal.ErrIndexNotFound",
    L.ERR_WRONG_TYPE: "proto.ErrWrongType",
    L.ERR_UNEXPECTED_TYPE: "unexpected block type",
    L.ERR_FILE_NOT_FOUND: "wal.ErrFileNotFound",
}

metadataType, entryType, stateType, crcType = 1, 2, 3, 4


@dataclass
class HardState:
    """raftpb.HardState, raft/raftpb/raft.pb.go:143-148"""
    Term: int = 0
    Vote: int = 0
    Commit: int = 0
    XXX_unrecognized: Optional[bytes] = None


@dataclass
class Entry:
    """raftpb.Entry, raft/raftpb/raft.pb.go:100-106 (Data None == Go nil)"""
    Type: int = 0
    Term: int = 0
    Index: int = 0
    Data: Optional[bytes] = None
    XXX_unrecognized: Optional[bytes] = None


_live = weakref.WeakSet()


@atexit.register
def _close_all():
    """every ctx still open at interpreter exit is destroyed before the HIP
    runtime's own teardown (a ctx's CU-masked streams must go first)"""
    for c in list(_live):
        try:
            c.close()
        except Exception:
            pass


class Context:
    """One GPU context (device workspace + stream), ewal_ctx_create."""

    def __init__(self, device=0):
        self._p = C.c_void_p()
        check(lib.ewal_ctx_create(device, C.byref(self._p)))
        self.device = device
        _live.add(self)

    @property
    def handle(self):
        return self._p

    def close(self):
        if self._p:
            lib.ewal_ctx_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_options(self, general_path=False, overlap=False, vh=None):
        """ewal_ctx_set_options: general_path=True makes every ReadAll take the
        general path (for cross-checking it against the fused pass);
        overlap=True the opt-in overlapped stream / frame pipeline; vh=True /
        False forces the frame pass's 128-B prefixes on / off (None: on for
        record-dense WALs)."""
        check(lib.ewal_ctx_set_options(self._p, (L.OPT_GENERAL_PATH if general_path else 0) |
                                       (L.OPT_OVERLAP if overlap else 0) |
                                       (0 if vh is None else (L.OPT_VH_ON if vh else L.OPT_VH_OFF))))

    def set_stream(self, hip_stream):
        """Run this ctx's work on a caller-owned hipStream_t (e.g. torch's)."""
        check(lib.ewal_ctx_set_stream(self._p, C.c_void_p(hip_stream)))

    def alloc(self, n):
        d = C.c_void_p()
        check(lib.ewal_device_alloc(self._p, n, C.byref(d)))
        return DeviceBuffer(self, d, n)


class DeviceBuffer:
    """Device memory owned through the library (ewal_device_alloc)."""

    def __init__(self, ctx, ptr, n):
        self.ctx, self.ptr, self.n = ctx, ptr, n

    def upload(self, data, offset=0):
        b = bytes(data) if not isinstance(data, (bytes, bytearray)) else data
        # zero-copy views of the host bytes (the copy only reads them)
        src = C.c_char_p(b) if isinstance(b, bytes) else (C.c_char * len(b)).from_buffer(b)
        check(lib.ewal_upload(self.ctx.handle, C.c_void_p(self.ptr.value + offset), src, len(b)))

    def upload_ptr(self, host_ptr, n, offset=0):
        check(lib.ewal_upload(self.ctx.handle, C.c_void_p(self.ptr.value + offset), C.c_void_p(host_ptr), n))

    def download(self, n=None, offset=0):
        n = self.n if n is None else n
        out = (C.c_char * n)()
        check(lib.ewal_download(self.ctx.handle, out, C.c_void_p(self.ptr.value + offset), n))
        return out.raw

    def free(self):
        if self.ptr:
            lib.ewal_device_free(self.ctx.handle, self.ptr)
            self.ptr = C.c_void_p()


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


@dataclass
class ReadAllResult:
    status: int
    detail: int
    fail_record: int
    fail_offset: int
    n_records: int
    last_crc: int
    enti: int
    metadata: Optional[bytes]
    state: HardState
    ents: List[Entry] = field(default_factory=list)
    n_candidates: int = 0
    n_runs: int = 0
    device_ms: float = 0.0
    stream_ms: float = 0.0
    n_slow: int = 0           # frames decoded by the general (non-canonical) walker
    flags: int = 0            # FLAG_SHARD_FALLBACK: a batched shard verified on its own

    def as_dict(self):
        return dict(status=self.status, detail=self.detail, fail_record=self.fail_record,
                    fail_offset=self.fail_offset, n_records=self.n_records, last_crc=self.last_crc, enti=self.enti,
                    metadata=self.metadata, state=dict(term=self.state.Term, vote=self.state.Vote,
                                                       commit=self.state.Commit,
                                                       unrec=self.state.XXX_unrecognized),
                    ents=[dict(type=e.Type, term=e.Term, index=e.Index, data=e.Data, unrec=e.XXX_unrecognized)
                          for e in self.ents])


def split_bytes(ctx, shard=None) -> bytes:
    """The side bytes the last ReadAll gathered on the device for split byte
    fields (Record.Data / Entry.Data repeated with several non-empty
    segments): data_nil == 2 ents and EWAL_FLAG_METADATA_SPLIT metadata index
    them (ewal_copy_split_bytes; a batched shard's: ewal_batch_copy_split_bytes)."""
    if shard is None:
        n = lib.ewal_copy_split_bytes(ctx.handle, None, 0)
    else:
        n = lib.ewal_batch_copy_split_bytes(ctx.handle, shard, None, 0)
    check(0 if n >= 0 else int(n))
    raw = (C.c_char * max(n, 1))()
    if n:
        got = (lib.ewal_copy_split_bytes(ctx.handle, raw, n) if shard is None
               else lib.ewal_batch_copy_split_bytes(ctx.handle, shard, raw, n))
        check(0 if got >= 0 else int(got))
    return raw.raw[:n]


def _collect(ctx, r, buf_view, with_ents=True, shard=None):
    ok = r.status == L.OK
    md = None
    side = None                # the split bytes, fetched when a view needs them
    if ok and r.metadata_off >= 0:
        if r.flags & L.FLAG_METADATA_SPLIT:
            side = split_bytes(ctx, shard)
            md = side[r.metadata_off:r.metadata_off + r.metadata_len]
        else:
            md = bytes(buf_view[r.metadata_off:r.metadata_off + r.metadata_len])
    st = HardState(r.state_term, r.state_vote, r.state_commit) if (ok and r.has_state) else HardState()
    ents = []
    if ok and with_ents and r.n_ents:
        arr = (L.EntryDesc * r.n_ents)()
        if shard is None:
            n = lib.ewal_copy_entries(ctx.handle, arr, r.n_ents)
        else:
            n = lib.ewal_batch_copy_entries(ctx.handle, shard, arr, r.n_ents)
        check(0 if n >= 0 else int(n))
        for e in arr[:n]:
            if e.data_nil == 2:    # a range of the split bytes
                if side is None:
                    side = split_bytes(ctx, shard)
                data = side[e.data_off:e.data_off + e.data_len]
            else:
                data = None if e.data_nil else bytes(buf_view[e.data_off:e.data_off + e.data_len])
            ents.append(Entry(e.type, e.term, e.index, data))
    if ok and r.n_unrec:
        for ent, b in unrecognized(ctx, r.n_unrec, shard):
            if ent < 0:
                st.XXX_unrecognized = b
            elif ent < len(ents):
                ents[ent].XXX_unrecognized = b
    # last_crc: Go's lastCRC on success; kept with ErrIndexNotFound too (a split WAL's next range starts from it)
    keep_crc = ok or r.status == L.ERR_INDEX_NOT_FOUND
    return ReadAllResult(r.status, r.detail, r.fail_record, r.fail_offset, r.n_records, r.last_crc if keep_crc else 0,
                         r.enti, md, st, ents, r.n_candidates, r.n_runs, r.device_ms, r.stream_ms, r.n_slow,
                         r.flags)


def unrecognized(ctx, n, shard=None):
    """The last ReadAll's XXX_unrecognized side list: [(ent index or -1 for
    the HardState, bytes)] (ewal_copy_unrec / ewal_copy_unrec_bytes; a
    batched shard's: ewal_batch_copy_unrec / _bytes)."""
    arr = (L.UnrecDesc * max(n, 1))()
    if shard is None:
        k = lib.ewal_copy_unrec(ctx.handle, arr, n)
    else:
        k = lib.ewal_batch_copy_unrec(ctx.handle, shard, arr, n)
    check(0 if k >= 0 else int(k))
    tot = max([a.off + a.len for a in arr[:k]] + [0])
    raw = (C.c_char * max(tot, 1))()
    if shard is None:
        got = lib.ewal_copy_unrec_bytes(ctx.handle, raw, tot)
    else:
        got = lib.ewal_batch_copy_unrec_bytes(ctx.handle, shard, raw, tot)
    check(0 if got >= 0 else int(got))
    return [(a.ent, raw.raw[a.off:a.off + a.len]) for a in arr[:k]]


def readall_bytes(buf: bytes, ri: int = 0, ctx: Context = None, with_ents=True) -> ReadAllResult:
    """ReadAll over the concatenated WAL bytes (host memory, staged to HBM)."""
    ctx = ctx or default_context()
    r = L.Result()
    b = bytes(buf)
    rc = lib.ewal_readall_host(ctx.handle, b, len(b), ri, C.byref(r))
    if rc < 0:
        check(rc)
    return _collect(ctx, r, memoryview(b), with_ents)


def readall_device(dbuf: DeviceBuffer, n: int, ri: int = 0, host_view=None, with_ents=False) -> ReadAllResult:
    """ReadAll over WAL bytes already resident in HBM."""
    r = L.Result()
    rc = lib.ewal_readall_device(dbuf.ctx.handle, dbuf.ptr, n, ri, C.byref(r))
    if rc < 0:
        check(rc)
    return _collect(dbuf.ctx, r, host_view if host_view is not None else b"", with_ents and host_view is not None)


def readall_range_device(dbuf: DeviceBuffer, n: int, ri: int = 0, defer_first=True, host_view=None,
                         with_ents=False) -> ReadAllResult:
    """ReadAll over one range of a WAL split inside a file (ewal_readall_range_device):
    with defer_first, frame 0's CRC check is left to the caller (range_info's
    first_* operands; shard.split_verdict makes it)."""
    r = L.Result()
    rc = lib.ewal_readall_range_device(dbuf.ctx.handle, dbuf.ptr, n, ri, L.RANGE_DEFER_FIRST if defer_first else 0,
                                       C.byref(r))
    if rc < 0:
        check(rc)
    return _collect(dbuf.ctx, r, host_view if host_view is not None else b"", with_ents and host_view is not None)


def range_probe(dbuf: DeviceBuffer, n: int, start: int, window: int = 1 << 20):
    """(first frame-start candidate at or after start, Index of the first entry
    on the chain from it) of the n stream bytes in dbuf (ewal_range_probe);
    -1 for none."""
    pos, idx = C.c_int64(-1), C.c_int64(-1)
    check(lib.ewal_range_probe(dbuf.ctx.handle, dbuf.ptr, n, start, window, C.byref(pos), C.byref(idx)))
    return pos.value, idx.value


def readall_batch_device(dbuf: DeviceBuffer, lens, ris, host_views=None, with_ents=False) -> List[ReadAllResult]:
    """ReadAll of every shard of a batch resident in HBM: shard s is the
    lens[s] bytes after shards 0..s-1 (ewal_readall_batch_device); one
    result per shard, as if each were replayed alone with w.ri = ris[s]."""
    ns = len(lens)
    out = (L.Result * max(ns, 1))()
    rc = lib.ewal_readall_batch_device(dbuf.ctx.handle, dbuf.ptr, ns, (C.c_uint64 * max(ns, 1))(*lens),
                                       (C.c_uint64 * max(ns, 1))(*ris), out)
    if rc < 0:
        check(rc)
    res = []
    for s in range(ns):
        hv = host_views[s] if host_views is not None else b""
        res.append(_collect(dbuf.ctx, out[s], hv, with_ents and host_views is not None, shard=s))
    return res


def readall_batch_bytes(shards, ris, ctx: Context = None, with_ents=True) -> List[ReadAllResult]:
    """Batched ReadAll over host byte strings (concatenated, staged to HBM)."""
    ctx = ctx or default_context()
    blob = b"".join(bytes(x) for x in shards)
    d = ctx.alloc(len(blob) + 64)
    try:
        if blob:
            d.upload(blob)
        return readall_batch_device(d, [len(x) for x in shards], ris, [memoryview(bytes(x)) for x in shards],
                                    with_ents)
    finally:
        d.free()


def records(ctx: Context, n: int):
    """Per-frame descriptors of the last ReadAll on ctx."""
    arr = (L.RecordDesc * max(n, 1))()
    k = lib.ewal_copy_records(ctx.handle, arr, n)
    check(0 if k >= 0 else int(k))
    return [dict(offset=x.offset, data_off=x.data_off, data_len=x.data_len, type=x.type, crc=x.crc,
                 chained_crc=x.chained_crc) for x in arr[:k]]


class NotFinal(RuntimeError):
    """A joined multi-range ReadAll whose verdict is not final: ranges
    `resplit`.. must be read joined (ewal_split_result.resplit), which the
    caller does when its device-resident ranges are not one contiguous span."""

    def __init__(self, resplit):
        super().__init__("joined verdict not final: read ranges %d.. joined" % resplit)
        self.resplit = resplit


class Multi:
    """ewal_multi: (*WAL).ReadAll over ONE WAL split across the contexts
    `ctxs` of this process (distinct ctxs; they may share a device), one host
    thread per ctx, returning ReadAll's whole result -- verdict, metadata,
    HardState and the ents joined across the ranges (wal/wal.go:164-216, the
    caller etcdserver/server.go:153-168)."""

    def __init__(self, ctxs):
        arr = (C.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
        h = C.c_void_p()
        check(lib.ewal_multi_create(arr, len(ctxs), C.byref(h)))
        self._h = h
        self.ctxs = list(ctxs)
        self.resplit = -1

    def close(self):
        if self._h:
            lib.ewal_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def readall(self, buf, ri=0, files=None, with_ents=True) -> ReadAllResult:
        """From host bytes; files = [(length, name index)] splits by file,
        None inside the stream (ranges at frame-start candidates)."""
        offs = idx = None
        nf = 0
        if files is not None:
            nf = len(files)
            o = [0]
            for n, _ in files:
                o.append(o[-1] + n)
            offs = (C.c_uint64 * (nf + 1))(*o)
            idx = (C.c_uint64 * nf)(*[i & ((1 << 64) - 1) for _, i in files])
        out = L.SplitResult()
        b = bytes(buf)
        rc = lib.ewal_multi_readall(self._h, b, len(b), offs, idx, nf, ri & ((1 << 64) - 1), C.byref(out))
        if rc < 0:
            check(rc)
        return self._result(out, memoryview(b), with_ents)

    def plan_device(self, dbuf: DeviceBuffer, n: int, ri=0):
        """ewal_multi_plan_device: range starts (n_ctx + 1) and w.ri per range
        of the device-resident stream dbuf[0, n)."""
        k = len(self.ctxs)
        st = (C.c_uint64 * (k + 1))()
        ris = (C.c_uint64 * k)()
        check(lib.ewal_multi_plan_device(self._h, dbuf.ptr, n, ri & ((1 << 64) - 1), st, ris))
        return list(st), list(ris)

    def readall_device(self, dbuf: DeviceBuffer, n: int, ri=0, plan=None, host_view=None,
                       with_ents=False) -> ReadAllResult:
        """Device-resident: range r = dbuf[starts[r], starts[r + 1]) read by
        ctx r in place (ewal_multi_readall_device); plan = plan_device's
        answer (computed here when None).  host_view: the same bytes on the
        host, for the ents' Data (with_ents)."""
        starts, ris = plan if plan is not None else self.plan_device(dbuf, n, ri)
        k = len(self.ctxs)
        base = dbuf.ptr.value if isinstance(dbuf.ptr, C.c_void_p) else int(dbuf.ptr)
        dr = (C.c_void_p * k)(*[base + starts[r] for r in range(k)])
        st = (C.c_uint64 * (k + 1))(*starts)
        rs = (C.c_uint64 * k)(*ris)
        out = L.SplitResult()
        rc = lib.ewal_multi_readall_device(self._h, dr, st, rs, None, ri & ((1 << 64) - 1), C.byref(out))
        if rc < 0:
            check(rc)
        return self._result(out, host_view, with_ents and host_view is not None)

    def timing(self):
        t = (C.c_double * 4)()
        check(lib.ewal_multi_timing(self._h, t))
        return dict(wall_ms=t[0], max_range_device_ms=t[1], join_ms=t[2], resplits=int(t[3]))

    def rows(self):
        k = len(self.ctxs)
        arr = (L.RangeRow * k)()
        st = (C.c_uint64 * k)()
        check(min(0, lib.ewal_multi_copy_rows(self._h, arr, st, k)))
        return list(arr), list(st)

    def _result(self, out, view, with_ents) -> ReadAllResult:
        self.resplit = out.resplit
        if out.resplit >= 0:
            # not a final verdict: device-resident ranges k.. are not one contiguous
            # device span, so the C driver handed the re-read back (ewal_multi_readall_device)
            raise NotFinal(out.resplit)
        ok = out.status == L.OK
        md = None
        if ok and out.md_range >= 0:
            n = max(out.md_len, 0)
            raw = (C.c_char * max(n, 1))()
            got = lib.ewal_multi_copy_metadata(self._h, raw, n)
            check(0 if got >= 0 else int(got))
            md = raw.raw[:n]
        st = HardState(out.state_term, out.state_vote, out.state_commit) if (ok and out.state_range >= 0) \
            else HardState()
        ents = []
        if ok and with_ents and out.n_ents:
            arr = (L.EntryDesc * out.n_ents)()
            n = lib.ewal_multi_copy_entries(self._h, arr, out.n_ents)
            check(0 if n >= 0 else int(n))
            side = None
            for e in arr[:n]:
                if e.data_nil == 2:
                    if side is None:
                        k = lib.ewal_multi_copy_split_bytes(self._h, None, 0)
                        raw = (C.c_char * max(k, 1))()
                        lib.ewal_multi_copy_split_bytes(self._h, raw, k)
                        side = raw.raw[:k]
                    data = side[e.data_off:e.data_off + e.data_len]
                else:
                    data = None if e.data_nil else bytes(view[e.data_off:e.data_off + e.data_len])
                ents.append(Entry(e.type, e.term, e.index, data))
        if ok:
            nu = lib.ewal_multi_copy_unrec(self._h, None, 0)
            check(0 if nu >= 0 else int(nu))
            if nu:
                arr = (L.UnrecDesc * nu)()
                lib.ewal_multi_copy_unrec(self._h, arr, nu)
                tot = lib.ewal_multi_copy_unrec_bytes(self._h, None, 0)
                raw = (C.c_char * max(tot, 1))()
                lib.ewal_multi_copy_unrec_bytes(self._h, raw, tot)
                for a in arr[:nu]:
                    b = raw.raw[a.off:a.off + a.len]
                    if a.ent < 0:
                        st.XXX_unrecognized = b
                    elif a.ent < len(ents):
                        ents[a.ent].XXX_unrecognized = b
        keep_crc = ok or out.status == L.ERR_INDEX_NOT_FOUND
        r = ReadAllResult(out.status, out.detail, out.fail_record, -1, out.n_records,
                          out.last_crc if keep_crc else 0, out.enti, md, st, ents)
        r.n_ents = out.n_ents
        return r


def readall_multi(ctxs, buf, ri=0, files=None, with_ents=True):
    """ewal_multi_readall through a one-call Multi: ReadAll over ONE WAL (host
    bytes `buf`) split across `ctxs`.  Returns (ReadAllResult, timing)."""
    m = Multi(ctxs)
    try:
        r = m.readall(buf, ri, files, with_ents)
        return r, m.timing()
    finally:
        m.close()


def range_info(ctx: Context, stream=None, dbuf: DeviceBuffer = None):
    """ewal_copy_range_info of the last ReadAll on ctx: what its range of ONE WAL
    split by file contributes to shard.split_verdict.  The metadata Data
    bytes are read from `stream` (host bytes of the range) or `dbuf` (its
    device buffer); None == Go nil."""
    ri = L.RangeInfo()
    check(lib.ewal_copy_range_info(ctx.handle, C.byref(ri)))

    def data(off, n, split):
        if off < 0:
            return None
        if split:   # a metadata Data in several segments: its concatenation, gathered on the device
            return split_bytes(ctx)[off:off + n]
        if stream is not None:
            return bytes(stream[off:off + n])
        return dbuf.download(n, off) if n else b""
    return dict(n_frames=ri.n_frames, first_crc=ri.first_crc, md_first_frame=ri.md_first_frame,
                md_first=data(ri.md_first_off, ri.md_first_len, ri.md_split & 1) if ri.md_first_frame >= 0 else None,
                md_value=data(ri.md_value_off, ri.md_value_len, ri.md_split & 2) if ri.md_value_frame >= 0 else None,
                md_value_frame=ri.md_value_frame, first_entry_frame=ri.first_entry_frame,
                first_entry_index=ri.first_entry_index, min_entry_index=ri.min_entry_index,
                last_entry_index=ri.last_entry_index, last_op_frame=ri.last_op_frame,
                last_op_index=ri.last_op_index, first_type=ri.first_type, first_dlen=ri.first_dlen,
                first_stored_crc=ri.first_stored_crc, first_u0=ri.first_u0, last_entry_frame=ri.last_entry_frame,
                first_pre_crc=ri.first_pre_crc, end_off=ri.end_off, n_bytes=ri.n_bytes,
                state_frame=ri.state_frame, state=(ri.state_term, ri.state_vote, ri.state_commit),
                state_unrec=ri.state_unrec)


class WAL:
    """wal.WAL opened for reading (OpenAtIndex) -- ReadAll runs on the GPU."""

    def __init__(self, handle, ctx):
        self._h, self._ctx = handle, ctx

    def ReadAll(self):
        if self._ctx is None:
            self._ctx = default_context()
        r = L.Result()
        rc = lib.ewal_wal_readall(self._h, self._ctx.handle, C.byref(r))
        if rc < 0:
            check(rc)
        n = C.c_uint64(0)
        p = lib.ewal_wal_bytes(self._h, C.byref(n))
        view = C.string_at(p, n.value) if n.value else b""
        res = _collect(self._ctx, r, memoryview(view))
        if res.status != L.OK:
            check(res.status, res.detail, res.fail_record, res.fail_offset)
        return res.metadata, res.state, res.ents

    @property
    def seq(self):
        return lib.ewal_wal_seq(self._h)

    def Close(self):
        if self._h:
            lib.ewal_wal_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.Close()
        except Exception:
            pass


def parseWalName(name: str):
    """(seq, index) of "%016x-%016x.wal", or raises ValueError (wal/util.go:77-84)."""
    s, i = C.c_uint64(), C.c_uint64()
    if not lib.ewal_parse_wal_name(name.encode(), C.byref(s), C.byref(i)):
        raise ValueError("bad wal name: %s" % name)
    return s.value, i.value


def _names(names):
    return (C.c_char_p * max(1, len(names)))(*[n.encode() for n in names])


def searchIndex(names, index):
    """(last i with parseWalName(names[i]).index <= index, found) (wal/util.go:20-32)."""
    k = lib.ewal_search_index(_names(names), len(names), index)
    if k < -1:
        check(int(k))
    return int(k), k >= 0


def isValidSeq(names):
    """The seqs of sorted names increase by one (the check skipped while the
    last seq is 0), wal/util.go:36-49."""
    r = lib.ewal_is_valid_seq(_names(names), len(names))
    if r < 0:
        check(r)
    return r == 1


def walName(seq, index):
    out = C.create_string_buffer(38)
    lib.ewal_wal_name(seq, index, out)
    return out.value.decode()


def OpenAtIndex(dirpath: str, index: int, ctx: Context = None) -> WAL:
    h = C.c_void_p()
    st = lib.ewal_open_at_index(dirpath.encode(), index, C.byref(h))
    check(st)
    return WAL(h, ctx)


class Writer:
    """wal.WAL in append mode (Create / Cut / Save*)."""

    def __init__(self, h):
        self._h = h

    def SaveEntry(self, e: Entry):
        check(lib.ewal_writer_save_entry(self._h, e.Type, e.Term, e.Index, e.Data or b"", len(e.Data or b"")))

    def SaveState(self, s: HardState):
        check(lib.ewal_writer_save_state(self._h, s.Term, s.Vote, s.Commit))

    def Save(self, st: HardState, ents: List[Entry]):
        self.SaveState(st)
        for e in ents:
            self.SaveEntry(e)
        self.Sync()

    def Cut(self):
        check(lib.ewal_writer_cut(self._h))

    def Sync(self):
        check(lib.ewal_writer_sync(self._h))

    def Close(self):
        if self._h:
            lib.ewal_writer_close(self._h)
            self._h = None


def Create(dirpath: str, metadata: Optional[bytes]) -> Writer:
    h = C.c_void_p()
    md = metadata or b""
    st = lib.ewal_create(dirpath.encode(), md, len(md), int(metadata is None), C.byref(h))
    if st == L.E_IO:
        raise FileExistsError(dirpath)
    check(st)
    return Writer(h)


class Encoder:
    """In-memory encoder.encode (wal/encoder.go:25-37)."""

    def __init__(self, prev_crc=0, reserve=0):
        self._h = lib.ewal_encoder_new(prev_crc, reserve)

    def encode(self, type_, data):
        d = data if data is not None else b""
        check(lib.ewal_encoder_encode(self._h, type_, d, len(d), int(data is None)))

    def save_entry(self, type_=0, term=0, index=0, data=None):
        d = data or b""
        check(lib.ewal_encoder_save_entry(self._h, type_, term, index, d, len(d)))

    def save_state(self, term=0, vote=0, commit=0):
        check(lib.ewal_encoder_save_state(self._h, term, vote, commit))

    def getvalue(self):
        n = C.c_uint64(0)
        p = lib.ewal_encoder_bytes(self._h, C.byref(n))
        return C.string_at(p, n.value) if n.value else b""

    @property
    def crc(self):
        return lib.ewal_encoder_crc(self._h)

    def __del__(self):
        try:
            lib.ewal_encoder_free(self._h)
        except Exception:
            pass


def encode_entries_device(ctx: Context, entries, prev_crc: int = 0):
    """SaveEntry for every entry, in order, on the GPU (encoder.encode,
    wal/wal.go:248-263, wal/encoder.go:25-37): returns (frame bytes, the
    chained CRC after the last entry) -- byte-identical to Encoder.save_entry
    in a loop."""
    payload = b"".join((e.Data or b"") for e in entries)
    n = len(entries)
    arr = (L.EntryDesc * max(1, n))()
    off = 0
    for i, e in enumerate(entries):
        d = e.Data or b""
        arr[i].term, arr[i].index, arr[i].data_off, arr[i].data_len = e.Term, e.Index, off, len(d)
        arr[i].type, arr[i].data_nil = e.Type, int(e.Data is None)
        off += len(d)
    cap = len(payload) + 80 * n + 64
    dd, de, do = ctx.alloc(len(payload) + 64), ctx.alloc(C.sizeof(arr)), ctx.alloc(cap)
    try:
        if payload:
            dd.upload(payload)
        de.upload(bytes(arr))
        out_len, crc = C.c_uint64(), C.c_uint32()
        check(lib.ewal_encode_entries_device(ctx.handle, dd.ptr, len(payload), de.ptr, n, prev_crc, do.ptr, cap,
                                             C.byref(out_len), C.byref(crc)))
        return (do.download(out_len.value) if out_len.value else b""), crc.value
    finally:
        for b in (dd, de, do):
            b.free()


def save_device(ctx: Context, ops, prev_crc: int = 0):
    """A sequence of (*WAL).SaveState / SaveEntry / Cut calls encoded on the
    GPU in one chained call (ewal_save_device; wal/wal.go:219-279).  ops:
    ("entry", Entry) | ("state", HardState) | ("cut", metadata bytes or None).
    Returns (frame bytes, the running CRC after the last op, the offset of
    each op's first frame)."""
    n = len(ops)
    arr = (L.SaveRec * max(1, n))()
    parts, off = [], 0
    for i, (kind, x) in enumerate(ops):
        r = arr[i]
        if kind == "entry":
            d = x.Data or b""
            r.kind, r.etype, r.a, r.b = L.SAVE_ENTRY, x.Type, x.Term, x.Index
        elif kind == "state":
            d = b""
            r.kind, r.a, r.b, r.c = L.SAVE_STATE, x.Term, x.Vote, x.Commit
        elif kind == "cut":
            d = x or b""
            r.kind, r.data_nil = L.SAVE_CUT, int(x is None)
        else:
            raise ValueError(kind)
        r.data_off, r.data_len = off, len(d)
        parts.append(d)
        off += len(d)
    payload = b"".join(parts)
    cap = len(payload) + 120 * n + 64
    dd, dr, do = ctx.alloc(len(payload) + 64), ctx.alloc(C.sizeof(arr)), ctx.alloc(cap)
    try:
        if payload:
            dd.upload(payload)
        dr.upload(bytes(arr))
        out_len, crc = C.c_uint64(), C.c_uint32()
        offs = (C.c_uint64 * max(1, n))()
        check(lib.ewal_save_device(ctx.handle, dd.ptr, len(payload), dr.ptr, n, prev_crc, do.ptr, cap,
                                   C.byref(out_len), C.byref(crc), offs))
        return (do.download(out_len.value) if out_len.value else b""), crc.value, list(offs[:n])
    finally:
        for b in (dd, dr, do):
            b.free()


def synth_wal(target_bytes, min_data=64, max_data=65536, seed=2, corrupt_record=-1, rewind_per_mille=0,
              last_index=None):
    """Synthetic WAL (bench/test input); returns (bytearray, n_records).
    rewind_per_mille: that share of the entries open a new leader's term that
    rewrites the last 1..8 indexes; last_index (a list) receives the last
    entry's Index."""
    cap = target_bytes + max_data * 2 + (1 << 20) + target_bytes // 128   # (term varints grow with rewinds)
    out = bytearray(cap)
    nrec = C.c_int64(0)
    li = C.c_uint64(0)
    n = L.synth_lib().ewal_synth_wal_ex(seed, target_bytes, min_data, max_data, corrupt_record, rewind_per_mille,
                              (C.c_char * cap).from_buffer(out), cap, C.byref(nrec), C.byref(li))
    if n < 0:
        check(int(n))
    del out[n:]
    if last_index is not None:
        last_index.append(li.value)
    return out, nrec.value


def synth_shards(seeds, target_bytes, min_data, max_data, corrupt=None):
    """Per-raft-group WAL shards laid end to end (bench/test input for the
    batched ReadAll): shard i = synth_wal(target_bytes, seed=seeds[i]),
    corrupt = {shard index: record ordinal}.  Returns (bytearray, lens,
    n_records)."""
    corrupt = corrupt or {}
    per = target_bytes + max_data * 2 + (1 << 20)
    out = bytearray(per * len(seeds))
    base = C.addressof((C.c_char * len(out)).from_buffer(out))
    lens, nrec, pos = [], [], 0
    for i, sd in enumerate(seeds):
        nr = C.c_int64(0)
        n = L.synth_lib().ewal_synth_wal(sd, target_bytes, min_data, max_data, corrupt.get(i, -1), C.c_void_p(base + pos),
                               per, C.byref(nr))
        if n < 0:
            check(int(n))
        lens.append(n)
        nrec.append(nr.value)
        pos += n
    del out[pos:]
    return out, lens, nrec

