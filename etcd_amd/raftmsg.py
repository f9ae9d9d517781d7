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


def _fetch(copy, handle, desc, total):
    arr = (desc * max(total, 1))()
    if total:
        k = copy(handle, 0, arr, total)
        check(0 if k >= 0 else int(k))
    return arr


def decode_messages(ctx, bodies):
    """Decode message bodies (bytes each): one dict per body, with every
    XXX_unrecognized, split bytes field and the Snapshot's Nodes /
    RemovedNodes assembled from the message's segments (include/ewal.h)."""
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
        ents = _fetch(lib.emsg_copy_entries, ctx.handle, L.EntryDesc, tot.value)
        nseg = out[n - 1].segs_first + out[n - 1].n_segs
        segs = _fetch(lib.emsg_copy_segments, ctx.handle, L.SegmentDesc, nseg)
    finally:
        d.free()
    res = []
    for m in out:
        bykind = {}
        for g in segs[m.segs_first:m.segs_first + m.n_segs]:
            bykind.setdefault((g.kind, g.ent), []).append(g)

        def cat(kind, ent=-1):
            gs = bykind.get((kind, ent))
            return b"".join(blob[g.off:g.off + g.len] for g in gs) if gs else None

        es = []
        for j, e in enumerate(ents[m.ents_first:m.ents_first + m.n_ents]):
            ei = j   # segments name the entry by its index within the message
            data = (cat(L.SEG_ENTRY_DATA, ei) if e.data_nil == 2 else
                    None if e.data_nil else blob[e.data_off:e.data_off + e.data_len])
            ur = cat(L.SEG_ENTRY_UNREC, ei)
            es.append(dict(type=e.type, term=e.term, index=e.index, data=data, unrec=ur,
                           unrec_len=len(ur) if ur else 0))
        sd = (cat(L.SEG_SNAP_DATA) if m.snap_data_off == -2 else
              None if m.snap_data_off < 0 else blob[m.snap_data_off:m.snap_data_off + m.snap_data_len])
        su = cat(L.SEG_SNAP_UNREC)
        res.append(dict(status=m.status, type=m.type, to=m.to, from_=m.from_, term=m.term, log_term=m.log_term,
                        index=m.index, commit=m.commit, reject=bool(m.reject), ents=es, unrec_len=m.unrec_len,
                        unrec=cat(L.SEG_UNREC),
                        snap=dict(data=sd, index=m.snap_index, term=m.snap_term, n_nodes=m.snap_n_nodes,
                                  n_removed=m.snap_n_removed, unrec=su, unrec_len=len(su) if su else 0,
                                  nodes=[g.off for g in bykind.get((L.SEG_SNAP_NODE, -1), [])],
                                  removed=[g.off for g in bykind.get((L.SEG_SNAP_REMOVED, -1), [])])))
    return res
