"""snap.Snapshotter host mirror (snap/snapshotter.go) over the GPU batch verify.

* `snapshot_marshal` / `snap_file` -- raftpb.Snapshot.MarshalTo
  (raft/raftpb/raft.pb.go:944-982) and Snapshotter.save's envelope
  (snap/snapshotter.go:46-60: crc32.Update(0, Castagnoli, b), snappb.Snapshot
  {Crc, Data}.Marshal, snap/snappb/snap.pb.go:158-176); the CRC is the host
  SSE4.2 path of libewal (ewal_crc32_update_host).
* `verify_packed` -- loadSnap's CRC check for many files at once
  (esnap_verify_packed; snap/snapshotter.go:76-111).
* `load_dir` -- Snapshotter.Load (newest first, tried failures renamed
  .broken; snap/snapshotter.go:62-74); `snap_names` -- snapNames.
* `snapshot` / `copy_field` -- the full decoded raftpb.Snapshot (Data over
  repeated fields, Nodes / RemovedNodes past 64, XXX_unrecognized).
"""
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


def snapshot_marshal(data=b"", nodes=(), index=0, term=0, removed=()):
    """raftpb.Snapshot{Data, Nodes, Index, Term, RemovedNodes}.Marshal()."""
    parts = [b"\x0a", _varint(len(data)), data]
    parts += [b"\x10" + _varint(n) for n in nodes]
    parts += [b"\x18", _varint(index), b"\x20", _varint(term)]
    parts += [b"\x28" + _varint(n) for n in removed]
    return b"".join(parts)


def snap_file(body, poly=L.CASTAGNOLI):
    """The bytes Snapshotter.save writes for a marshalled raftpb.Snapshot."""
    crc = lib.ewal_crc32_update_host(0, poly, body, len(body))
    return b"".join([b"\x08", _varint(crc), b"\x12", _varint(len(body)), body])


def verify_packed(dbuf, buf_len, offs, lens, poly=L.CASTAGNOLI):
    """loadSnap's CRC verdict for n files packed in one device buffer:
    (status[], stored_crc[], computed_crc[])."""
    n = len(offs)
    st = (C.c_int32 * max(n, 1))()
    sc = (C.c_uint32 * max(n, 1))()
    cc = (C.c_uint32 * max(n, 1))()
    rc = lib.esnap_verify_packed(dbuf.ctx.handle, dbuf.ptr, buf_len, (C.c_uint64 * max(n, 1))(*offs),
                                 (C.c_uint64 * max(n, 1))(*lens), n, poly, st, sc, cc)
    check(rc)
    return list(st[:n]), list(sc[:n]), list(cc[:n])


def copy_field(ctx, i, field):
    """esnap_copy_field: the full value of one raftpb.Snapshot field of file i
    of the last verify_packed / load_dir -- bytes (None when Go leaves it
    nil) for SNAP_FIELD_DATA / SNAP_FIELD_UNREC, a list of uint64 for
    SNAP_FIELD_NODES / SNAP_FIELD_REMOVED."""
    n = lib.esnap_copy_field(ctx.handle, i, field, None, 0)
    if n < 0:
        check(int(n))
    if field in (L.SNAP_FIELD_NODES, L.SNAP_FIELD_REMOVED):
        buf = (C.c_uint64 * max(n, 1))()
        check(min(0, int(lib.esnap_copy_field(ctx.handle, i, field, buf, n))))
        return list(buf[:n])
    if n == 0:
        return None
    buf = C.create_string_buffer(n)
    check(min(0, int(lib.esnap_copy_field(ctx.handle, i, field, buf, n))))
    return buf.raw[:n]


def snapshot(ctx, i):
    """The decoded raftpb.Snapshot of file i (status OK) as a dict shaped like
    the oracle's loadsnap()["snap"], plus its XXX_unrecognized bytes."""
    s = L.SnapshotDesc()
    check(lib.esnap_copy_snapshot(ctx.handle, i, C.byref(s)))
    return dict(data=copy_field(ctx, i, L.SNAP_FIELD_DATA), nodes=copy_field(ctx, i, L.SNAP_FIELD_NODES),
                index=s.index, term=s.term, removed=copy_field(ctx, i, L.SNAP_FIELD_REMOVED),
                unrec=copy_field(ctx, i, L.SNAP_FIELD_UNREC))


def load_dir(ctx, dirpath, poly=L.CASTAGNOLI):
    """Snapshotter.Load(): (file name, esnap_snapshot) or raises EwalError."""
    s = L.SnapshotDesc()
    name = C.c_char_p()
    check(lib.esnap_load_dir(ctx.handle, dirpath.encode(), poly, C.byref(s), C.byref(name)))
    return name.value.decode(), s


def snap_names(dirpath):
    """Snapshotter.snapNames: *.snap names newest first; raises EwalError
    (ErrNoSnapshot) when there are none (snap/snapshotter.go:115-131)."""
    need = C.c_uint64(0)
    n = lib.esnap_names(dirpath.encode(), None, 0, C.byref(need))
    if n < 0:
        check(int(n))
    if n == 0:
        check(L.ERR_NO_SNAPSHOT)
    buf = C.create_string_buffer(max(1, need.value))
    lib.esnap_names(dirpath.encode(), buf, need.value, C.byref(need))
    return buf.raw[:need.value].decode().split("\0")[:n]
