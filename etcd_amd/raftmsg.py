"""raftpb.Message ingress decode on the GPU (emsg_decode_batch_device).

Mirrors `(*raftpb.Message).Unmarshal` (raft/raftpb/raft.pb.go:407-617), the
call etcdhttp's serveRaft makes for every POST /raft body
(etcdserver/etcdhttp/http.go:119-146), batched over many bodies.  Results are
dicts shaped like the oracle's `message_unmarshal` (tests compare them)."""
import ctypes as C

from . import _lib as L
from ._lib import lib, check


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def entry_marshal(type_=0, term=0, index=0, data=None):
    """raftpb.Entry.MarshalTo (raft/raftpb/raft.pb.go:921-943): field 4 always written."""
    d = data or b""
    return b"".join([b"\x08", _varint(type_ & 0xFFFFFFFFFFFFFFFF), b"\x10", _varint(term), b"\x18", _varint(index),
                     b"\x22", _varint(len(d)), d])


def message_marshal(type_=0, to=0, from_=0, term=0, log_term=0, index=0, entries=(), commit=0, snapshot=b"",
                    reject=False):
    """raftpb.Message.MarshalTo (raft/raftpb/raft.pb.go:1010-1068); entries are
    marshalled Entry bodies, snapshot a marshalled raftpb.Snapshot."""
    parts = [b"\x08", _varint(type_), b"\x10", _varint(to), b"\x18", _varint(from_), b"\x20", _varint(term),
             b"\x28", _varint(log_term), b"\x30", _varint(index)]
    for e in entries:
        parts += [b"\x3a", _varint(len(e)), e]
    parts += [b"\x40", _varint(commit), b"\x4a", _varint(len(snapshot)), snapshot, b"\x50",
              b"\x01" if reject else b"\x00"]
    return b"".join(parts)


def decode_messages(ctx, bodies):
    """Decode message bodies (bytes each): one dict per body."""
    n = len(bodies)
    if n == 0:
        return []
    blob = b"".join(bytes(b) for b in bodies)
    offs, pos = [], 0
    for b in bodies:
        offs.append(pos)
        pos += len(b)
    d = ctx.alloc(len(blob) + 64)
    try:
        if blob:
            d.upload(blob)
        out = (L.MessageDesc * n)()
        tot = C.c_uint64(0)
        check(lib.emsg_decode_batch_device(ctx.handle, d.ptr, len(blob), (C.c_uint64 * n)(*offs),
                                           (C.c_uint64 * n)(*[len(b) for b in bodies]), n, out, C.byref(tot)))
        ents = (L.EntryDesc * max(tot.value, 1))()
        if tot.value:
            k = lib.emsg_copy_entries(ctx.handle, 0, ents, tot.value)
            check(0 if k >= 0 else int(k))
    finally:
        d.free()
    res = []
    for m in out:
        es = [dict(type=e.type, term=e.term, index=e.index,
                   data=None if e.data_nil else blob[e.data_off:e.data_off + e.data_len])
              for e in ents[m.ents_first:m.ents_first + m.n_ents]]
        sd = None if m.snap_data_off < 0 else blob[m.snap_data_off:m.snap_data_off + m.snap_data_len]
        res.append(dict(status=m.status, type=m.type, to=m.to, from_=m.from_, term=m.term, log_term=m.log_term,
                        index=m.index, commit=m.commit, reject=bool(m.reject), ents=es, unrec_len=m.unrec_len,
                        snap=dict(data=sd, index=m.snap_index, term=m.snap_term, n_nodes=m.snap_n_nodes,
                                  n_removed=m.snap_n_removed)))
    return res
