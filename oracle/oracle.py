"""ctypes bindings for the CPU oracle (oracle/libewal_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product (etcd_amd/).  The C code
restates the reference's Go functions; see ewal_oracle.h for citations.
"""
import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libewal_oracle.so")

OK, EOF, ERR_UNEXPECTED_EOF, ERR_RECORD_CRC, ERR_WAL_CRC = 0, 1, 2, 3, 4
ERR_METADATA_CONFLICT, ERR_INDEX_NOT_FOUND, ERR_WRONG_TYPE, ERR_UNEXPECTED_TYPE = 5, 6, 7, 8
ERR_FILE_NOT_FOUND, ERR_SNAP_CRC, ERR_NO_SNAPSHOT = 9, 10, 11
PANIC_NEG_LENGTH, PANIC_BOUNDS, PANIC_ENTRY, PANIC_STATE, PANIC_INDEX_GAP, NONTERMINATING = 32, 33, 34, 35, 36, 37

CASTAGNOLI, IEEE, KOOPMAN = 0x82F63B78, 0xEDB88320, 0xEB31D82E


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    if not os.path.exists(_LIB):
        build()
    return C.CDLL(_LIB)


lib = _load()
u8p = C.POINTER(C.c_uint8)


class Record(C.Structure):
    _fields_ = [("type", C.c_int64), ("crc", C.c_uint32), ("data", u8p), ("data_len", C.c_int64),
                ("unrec_len", C.c_int64)]


class Entry(C.Structure):
    _fields_ = [("type", C.c_int32), ("term", C.c_uint64), ("index", C.c_uint64), ("data", u8p),
                ("data_len", C.c_int64), ("unrec_len", C.c_int64), ("unrec", u8p)]


class HardState(C.Structure):
    _fields_ = [("term", C.c_uint64), ("vote", C.c_uint64), ("commit", C.c_uint64), ("unrec_len", C.c_int64),
                ("unrec", u8p)]


class Snapshot(C.Structure):
    _fields_ = [("data", u8p), ("data_len", C.c_int64), ("nodes", C.POINTER(C.c_uint64)), ("n_nodes", C.c_int64),
                ("index", C.c_uint64), ("term", C.c_uint64), ("removed", C.POINTER(C.c_uint64)),
                ("n_removed", C.c_int64), ("unrec_len", C.c_int64), ("unrec", u8p)]


class ReadAllResult(C.Structure):
    _fields_ = [("status", C.c_int), ("detail", C.c_int64), ("fail_record", C.c_int64), ("fail_offset", C.c_int64),
                ("n_records", C.c_int64), ("last_crc", C.c_uint32), ("enti", C.c_uint64), ("metadata", u8p),
                ("metadata_len", C.c_int64), ("state", HardState), ("has_state", C.c_int),
                ("ents", C.POINTER(Entry)), ("n_ents", C.c_int64)]


class Encoder(C.Structure):
    _fields_ = [("buf", u8p), ("len", C.c_int64), ("cap", C.c_int64), ("crc", C.c_uint32)]


class Decoder(C.Structure):
    _fields_ = [("buf", u8p), ("len", C.c_int64), ("pos", C.c_int64), ("crc", C.c_uint32)]


class LoadSnapResult(C.Structure):
    _fields_ = [("status", C.c_int), ("stored_crc", C.c_uint32), ("computed_crc", C.c_uint32), ("snap", Snapshot)]


lib.or_crc32_update.restype = C.c_uint32
lib.or_crc32_update.argtypes = [C.c_uint32, C.c_uint32, C.c_char_p, C.c_size_t]
lib.or_crc32_update_table.restype = C.c_uint32
lib.or_crc32_update_table.argtypes = [C.c_uint32, C.c_uint32, C.c_char_p, C.c_size_t]
lib.or_readall.argtypes = [C.c_char_p, C.c_int64, C.c_uint64, C.POINTER(ReadAllResult)]
lib.or_readall_free.argtypes = [C.POINTER(ReadAllResult)]
lib.or_encoder_init.argtypes = [C.POINTER(Encoder), C.c_uint32]
lib.or_encode.argtypes = [C.POINTER(Encoder), C.c_int64, C.c_char_p, C.c_int64, C.c_int]
lib.or_encoder_free.argtypes = [C.POINTER(Encoder)]
lib.or_decoder_init.argtypes = [C.POINTER(Decoder), C.c_char_p, C.c_int64]
lib.or_decode.argtypes = [C.POINTER(Decoder), C.POINTER(Record)]
lib.or_record_free.argtypes = [C.POINTER(Record)]
lib.or_entry_free.argtypes = [C.POINTER(Entry)]
lib.or_hardstate_free.argtypes = [C.POINTER(HardState)]
for _n, _t in (("record", Record), ("entry", Entry), ("hardstate", HardState), ("snapshot", Snapshot)):
    getattr(lib, "or_%s_unmarshal" % _n).argtypes = [C.c_char_p, C.c_int64, C.POINTER(_t)]
lib.or_proto_skip.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
lib.or_record_marshal.restype = C.c_int64
lib.or_record_marshal.argtypes = [C.c_int64, C.c_uint32, C.c_char_p, C.c_int64, C.c_int, C.c_char_p]
lib.or_entry_marshal.restype = C.c_int64
lib.or_entry_marshal.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, C.c_char_p, C.c_int64, C.c_char_p]
lib.or_hardstate_marshal.restype = C.c_int64
lib.or_hardstate_marshal.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_char_p]
lib.or_snapshot_marshal.restype = C.c_int64
lib.or_snapshot_marshal.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_uint64), C.c_int64, C.c_uint64, C.c_uint64,
                                    C.POINTER(C.c_uint64), C.c_int64, C.c_char_p]
lib.or_snappb_marshal.restype = C.c_int64
lib.or_snappb_marshal.argtypes = [C.c_uint32, C.c_char_p, C.c_int64, C.c_int, C.c_char_p]
lib.or_loadsnap.argtypes = [C.c_char_p, C.c_int64, C.c_uint32, C.POINTER(LoadSnapResult)]
lib.or_loadsnap_free.argtypes = [C.POINTER(LoadSnapResult)]
lib.or_maybe_commit.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_uint64, C.POINTER(C.c_uint64),
                                C.POINTER(C.c_uint64), C.c_uint64, C.c_uint64]
lib.or_ents_digest.restype = C.c_uint32
lib.or_ents_digest.argtypes = [C.POINTER(ReadAllResult)]
lib.or_ent_views_digest.restype = C.c_uint32
lib.or_ent_views_digest.argtypes = [C.c_char_p, C.c_void_p, C.c_int64]
lib.orf_crc32c_update.restype = C.c_uint32
lib.orf_crc32c_update.argtypes = [C.c_uint32, C.c_char_p, C.c_uint64]
lib.orf_readall.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_int, C.c_void_p]
lib.orf_result_free.argtypes = [C.c_void_p]
lib.orf_readall_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_uint64, C.c_int, C.c_void_p,
                                  C.c_void_p]
lib.orf_readall_batch_faithful.argtypes = lib.orf_readall_batch.argtypes
lib.orf_snap_verify_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p,
                                      C.c_void_p]
lib.orf_maybe_commit_batch.argtypes = [C.c_uint64] + [C.c_void_p] * 9 + [C.c_int]
lib.or_chain_crcs.restype = C.c_int64
lib.or_chain_crcs.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_uint32), C.c_int64, C.POINTER(C.c_int64)]


def _bytes(p, n):
    """Go []byte view: None for nil."""
    if not p:
        return None
    return C.string_at(p, n)


def crc32_update(crc, data, poly=CASTAGNOLI):
    return lib.or_crc32_update(crc, poly, bytes(data), len(data))


def crc32_update_table(crc, data, poly=CASTAGNOLI):
    return lib.or_crc32_update_table(crc, poly, bytes(data), len(data))


def _marshal(fn, *args):
    n = fn(*args, None)
    out = C.create_string_buffer(max(n, 1))
    fn(*args, out)
    return out.raw[:n]


def record_marshal(type_, crc, data):
    return _marshal(lib.or_record_marshal, type_, crc, data or b"", len(data or b""), int(data is None))


def entry_marshal(type_=0, term=0, index=0, data=None):
    d = data or b""
    return _marshal(lib.or_entry_marshal, type_, term, index, d, len(d))


def hardstate_marshal(term=0, vote=0, commit=0):
    return _marshal(lib.or_hardstate_marshal, term, vote, commit)


def snapshot_marshal(data=b"", nodes=(), index=0, term=0, removed=()):
    na = (C.c_uint64 * max(len(nodes), 1))(*nodes)
    ra = (C.c_uint64 * max(len(removed), 1))(*removed)
    return _marshal(lib.or_snapshot_marshal, data, len(data), na, len(nodes), index, term, ra, len(removed))


def snappb_marshal(crc, data):
    return _marshal(lib.or_snappb_marshal, crc, data or b"", len(data or b""), int(data is None))


def record_unmarshal(b):
    r = Record()
    st = lib.or_record_unmarshal(b, len(b), C.byref(r))
    out = dict(type=r.type, crc=r.crc, data=_bytes(r.data, r.data_len), unrec_len=r.unrec_len)
    lib.or_record_free(C.byref(r))
    return st, out


def entry_unmarshal(b):
    e = Entry()
    st = lib.or_entry_unmarshal(b, len(b), C.byref(e))
    out = dict(type=e.type, term=e.term, index=e.index, data=_bytes(e.data, e.data_len), unrec_len=e.unrec_len,
               unrec=_bytes(e.unrec, e.unrec_len))
    lib.or_entry_free(C.byref(e))
    return st, out


def hardstate_unmarshal(b):
    h = HardState()
    st = lib.or_hardstate_unmarshal(b, len(b), C.byref(h))
    out = dict(term=h.term, vote=h.vote, commit=h.commit, unrec=_bytes(h.unrec, h.unrec_len))
    lib.or_hardstate_free(C.byref(h))
    return st, out


def proto_skip(b):
    n = C.c_int64(0)
    st = lib.or_proto_skip(b, len(b), C.byref(n))
    return st, n.value


def decode(buf):
    """Drive decoder.decode over buf; list of (status, record dict, crc)."""
    d = Decoder()
    lib.or_decoder_init(C.byref(d), buf, len(buf))
    r = Record()
    out = []
    while True:
        st = lib.or_decode(C.byref(d), C.byref(r))
        out.append((st, dict(type=r.type, crc=r.crc, data=_bytes(r.data, r.data_len)), d.crc))
        if st != OK:
            break
    lib.or_record_free(C.byref(r))
    return out


def readall(buf, ri=0):
    """(*WAL).ReadAll over the concatenated files; returns a dict."""
    r = ReadAllResult()
    lib.or_readall(buf, len(buf), ri, C.byref(r))
    out = dict(status=r.status, detail=r.detail, fail_record=r.fail_record, fail_offset=r.fail_offset,
               n_records=r.n_records, last_crc=r.last_crc, enti=r.enti,
               metadata=_bytes(r.metadata, r.metadata_len),
               state=dict(term=r.state.term, vote=r.state.vote, commit=r.state.commit,
                          unrec=_bytes(r.state.unrec, r.state.unrec_len)) if r.has_state else
               dict(term=0, vote=0, commit=0, unrec=None),
               ents=[dict(type=r.ents[i].type, term=r.ents[i].term, index=r.ents[i].index,
                          data=_bytes(r.ents[i].data, r.ents[i].data_len),
                          unrec=_bytes(r.ents[i].unrec, r.ents[i].unrec_len)) for i in range(r.n_ents)])
    lib.or_readall_free(C.byref(r))
    return out


def readall_digest(buf, ri=0):
    """readall() for large inputs: the ents as (count, digest) instead of a
    list (or_ents_digest; test-side helper, not a restatement)."""
    r = ReadAllResult()
    lib.or_readall(buf, len(buf), ri, C.byref(r))
    out = dict(status=r.status, detail=r.detail, fail_record=r.fail_record, fail_offset=r.fail_offset,
               n_records=r.n_records, last_crc=r.last_crc, enti=r.enti,
               metadata=_bytes(r.metadata, r.metadata_len),
               state=(r.state.term, r.state.vote, r.state.commit) if r.has_state else (0, 0, 0),
               n_ents=r.n_ents, ents_digest=lib.or_ents_digest(C.byref(r)))
    lib.or_readall_free(C.byref(r))
    return out


def ent_views_digest(buf, views, n):
    """The same digest over n ewal_entry descriptors (ctypes array) into buf."""
    return lib.or_ent_views_digest(buf, C.cast(views, C.c_void_p), n)


# ---- the optimised CPU baseline (ewal_cpu_fast.c; bench.py's cpu_baseline) ----
IRREGULAR = 100


class FastEnt(C.Structure):
    _fields_ = [("term", C.c_uint64), ("index", C.c_uint64), ("data_off", C.c_uint64), ("data_len", C.c_uint64),
                ("type", C.c_int32), ("data_nil", C.c_int32)]


class FastResult(C.Structure):
    _fields_ = [("status", C.c_int), ("detail", C.c_int64), ("fail_record", C.c_int64), ("fail_offset", C.c_int64),
                ("n_records", C.c_int64), ("last_crc", C.c_uint32), ("enti", C.c_uint64),
                ("metadata_off", C.c_int64), ("metadata_len", C.c_int64), ("has_state", C.c_int),
                ("state_term", C.c_uint64), ("state_vote", C.c_uint64), ("state_commit", C.c_uint64),
                ("ents", C.POINTER(FastEnt)), ("n_ents", C.c_int64)]


def fast_crc32c(crc, data):
    return lib.orf_crc32c_update(crc, data, len(data))


def fast_readall(buf, ri=0, nthreads=1):
    """orf_readall: readall_digest()'s dict, or None when the input is
    outside the fast path (ORF_IRREGULAR)."""
    r = FastResult()
    keep = C.create_string_buffer(bytes(buf), len(buf))
    st = lib.orf_readall(C.addressof(keep), len(buf), ri, nthreads, C.byref(r))
    if st == IRREGULAR:
        return None
    md = buf[r.metadata_off:r.metadata_off + r.metadata_len] if r.metadata_off >= 0 else None
    out = dict(status=r.status, detail=r.detail, fail_record=r.fail_record, fail_offset=r.fail_offset,
               n_records=r.n_records, last_crc=r.last_crc, enti=r.enti, metadata=md,
               state=(r.state_term, r.state_vote, r.state_commit) if r.has_state else (0, 0, 0),
               n_ents=r.n_ents, ents_digest=lib.or_ent_views_digest(keep, C.cast(r.ents, C.c_void_p), r.n_ents))
    lib.orf_result_free(C.byref(r))
    return out


def fast_readall_status(buf_addr, n, ri=0, nthreads=1):
    """orf_readall over n bytes at buf_addr: (status, n_records, fail_record)
    only (the bench's timed call)."""
    r = FastResult()
    st = lib.orf_readall(C.c_void_p(buf_addr), n, ri, nthreads, C.byref(r))
    out = (st, r.n_records, r.fail_record)
    lib.orf_result_free(C.byref(r))
    return out


def restart_file(path, ri, nthreads, faithful):
    """orf_restart_file: (status, frames, read ms, total ms) of a CPU restart
    (file read + ReadAll)."""
    fr, rm, tm = C.c_int64(0), C.c_double(0), C.c_double(0)
    st = lib.orf_restart_file(path.encode(), ri, nthreads, int(faithful), C.byref(fr), C.byref(rm), C.byref(tm))
    return st, fr.value, rm.value, tm.value


def fast_message_batch(buf_addr, offs, lens, nthreads):
    """orf_message_batch: the status of every message's Unmarshal."""
    n = len(offs)
    st = (C.c_int32 * max(n, 1))()
    lib.orf_message_batch(C.c_void_p(buf_addr), _u64arr(offs), _u64arr(lens), n, nthreads, st)
    return list(st[:n])


def _u64arr(x):
    return (C.c_uint64 * max(len(x), 1))(*x)


def fast_readall_batch(buf_addr, offs, lens, ri, nthreads, faithful=False):
    """orf_readall_batch (faithful: or_readall per shard) over shards at
    buf_addr (an address), one shard per worker: (status, frames)."""
    n = len(offs)
    st, fr = (C.c_int32 * max(n, 1))(), (C.c_int64 * max(n, 1))()
    fn = lib.orf_readall_batch_faithful if faithful else lib.orf_readall_batch
    fn(C.c_void_p(buf_addr), _u64arr(offs), _u64arr(lens), n, ri, nthreads, st, fr)
    return list(st[:n]), list(fr[:n])


def fast_snap_verify_batch(buf_addr, offs, lens, nthreads):
    n = len(offs)
    st, cc = (C.c_int32 * max(n, 1))(), (C.c_uint32 * max(n, 1))()
    lib.orf_snap_verify_batch(C.c_void_p(buf_addr), _u64arr(offs), _u64arr(lens), n, nthreads, st, cc)
    return list(st[:n]), list(cc[:n])


def fast_maybe_commit_batch(G, match, nvoters, term, committed, log_offset, log_ptr, log_terms, changed, status,
                            nthreads):
    P = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731  (numpy arrays)
    lib.orf_maybe_commit_batch(G, P(match), P(nvoters), P(term), P(committed), P(log_offset), P(log_ptr),
                               P(log_terms), P(changed), P(status), nthreads)


def chain_crcs(buf, cap=None):
    cap = cap if cap is not None else max(1, len(buf) // 8)
    arr = (C.c_uint32 * cap)()
    offs = (C.c_int64 * cap)()
    n = lib.or_chain_crcs(buf, len(buf), arr, cap, offs)
    n = min(n, cap)
    return list(arr[:n]), list(offs[:n])


class WalEncoder:
    """encoder + the WAL record helpers (wal/encoder.go, wal/wal.go:256-292)."""

    def __init__(self, prev_crc=0):
        self._e = Encoder()
        lib.or_encoder_init(C.byref(self._e), prev_crc)

    def encode(self, type_, data):
        d = data if data is not None else b""
        lib.or_encode(C.byref(self._e), type_, d, len(d), int(data is None))

    def save_crc(self, prev_crc):           # wal/wal.go:290-292
        self.encode(4, None)

    def save_entry(self, type_=0, term=0, index=0, data=None):   # wal/wal.go:256-267
        self.encode(2, entry_marshal(type_, term, index, data))

    def save_state(self, term=0, vote=0, commit=0):              # wal/wal.go:269-279
        if term == 0 and vote == 0 and commit == 0:
            return
        self.encode(3, hardstate_marshal(term, vote, commit))

    @property
    def crc(self):
        return self._e.crc

    def getvalue(self):
        return C.string_at(self._e.buf, self._e.len) if self._e.len else b""

    def __del__(self):
        try:
            lib.or_encoder_free(C.byref(self._e))
        except Exception:
            pass


def loadsnap(b, poly=CASTAGNOLI):
    r = LoadSnapResult()
    st = lib.or_loadsnap(b, len(b), poly, C.byref(r))
    s = r.snap
    out = dict(status=st, stored_crc=r.stored_crc, computed_crc=r.computed_crc)
    if st == OK:
        out["snap"] = dict(data=_bytes(s.data, s.data_len), nodes=[s.nodes[i] for i in range(s.n_nodes)],
                           index=s.index, term=s.term, removed=[s.removed[i] for i in range(s.n_removed)],
                           unrec=_bytes(s.unrec, s.unrec_len))
    lib.or_loadsnap_free(C.byref(r))
    return out


def maybe_commit(matches, term, committed, log_terms, offset=0):
    m = (C.c_uint64 * max(len(matches), 1))(*matches)
    lt = (C.c_uint64 * max(len(log_terms), 1))(*log_terms)
    c = C.c_uint64(committed)
    rc = lib.or_maybe_commit(m, len(matches), term, C.byref(c), lt, len(log_terms), offset)
    return rc, c.value


lib.or_maybe_commit_batch.restype = None
lib.or_maybe_commit_batch.argtypes = [C.c_uint64] + [C.c_void_p] * 9


def maybe_commit_batch(G, match, nvoters, term, committed, log_offset, log_ptr, log_terms, changed, status):
    """or_maybe_commit_batch over numpy arrays (committed/changed/status written in place)."""
    ptr = lambda a: C.c_void_p(a.ctypes.data)   # noqa: E731
    lib.or_maybe_commit_batch(G, ptr(match), ptr(nvoters), ptr(term), ptr(committed), ptr(log_offset), ptr(log_ptr),
                              ptr(log_terms), ptr(changed), ptr(status))


# ---- raftpb.Message (raft/raftpb/raft.pb.go:407-617, 1010-1068) ----------
class Message(C.Structure):
    _fields_ = [("type", C.c_uint64), ("to", C.c_uint64), ("from_", C.c_uint64), ("term", C.c_uint64),
                ("log_term", C.c_uint64), ("index", C.c_uint64), ("commit", C.c_uint64), ("reject", C.c_int),
                ("ents", C.POINTER(Entry)), ("n_ents", C.c_int64), ("snap", Snapshot), ("unrec_len", C.c_int64),
                ("unrec", u8p)]


lib.or_message_unmarshal.argtypes = [C.c_char_p, C.c_int64, C.POINTER(Message)]
lib.or_message_free.argtypes = [C.POINTER(Message)]
lib.or_message_free.restype = None
lib.or_message_marshal.restype = C.c_int64
lib.or_message_marshal.argtypes = [C.c_uint64] * 6 + [C.c_char_p, C.POINTER(C.c_int64), C.c_int64, C.c_uint64,
                                                      C.c_char_p, C.c_int64, C.c_int, C.c_void_p]


def message_marshal(type_=0, to=0, from_=0, term=0, log_term=0, index=0, entries=(), commit=0, snapshot=b"",
                    reject=False):
    """entries: marshalled Entry bodies; snapshot: marshalled raftpb.Snapshot."""
    ents = b"".join(entries)
    lens = (C.c_int64 * max(len(entries), 1))(*[len(e) for e in entries])
    args = (type_, to, from_, term, log_term, index, ents, lens, len(entries), commit, snapshot, len(snapshot),
            int(bool(reject)))
    n = lib.or_message_marshal(*args, None)
    out = C.create_string_buffer(max(n, 1))
    lib.or_message_marshal(*args, out)
    return out.raw[:n]


def message_unmarshal(b):
    m = Message()
    st = lib.or_message_unmarshal(b, len(b), C.byref(m))
    ents = [dict(type=e.type, term=e.term, index=e.index, data=_bytes(e.data, e.data_len), unrec_len=e.unrec_len,
                 unrec=_bytes(e.unrec, e.unrec_len)) for e in m.ents[:m.n_ents]]
    s = m.snap
    out = dict(status=st, type=m.type, to=m.to, from_=m.from_, term=m.term, log_term=m.log_term, index=m.index,
               commit=m.commit, reject=bool(m.reject), ents=ents, unrec_len=m.unrec_len,
               unrec=_bytes(m.unrec, m.unrec_len),
               snap=dict(data=_bytes(s.data, s.data_len), index=s.index, term=s.term, n_nodes=s.n_nodes,
                         n_removed=s.n_removed, unrec_len=s.unrec_len, unrec=_bytes(s.unrec, s.unrec_len),
                         nodes=[s.nodes[i] for i in range(s.n_nodes)],
                         removed=[s.removed[i] for i in range(s.n_removed)]))
    lib.or_message_free(C.byref(m))
    return out

