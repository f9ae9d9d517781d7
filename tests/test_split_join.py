"""ewal_split_verdict (the C ABI join of ONE WAL read as several ranges,
etcd_amd/csrc/ewal_join.cpp) on rows built on the CPU: the oracle's per-range
ReadAll + range info for WALs split by file, and hand-made rows for the rules
the oracle cannot stand in for (a deferred frame 0 whose own read failed).
The join runs on the host: no GPU is needed."""
import random
import struct

from oracle import oracle as O
from etcd_amd import shard
from test_split_wal import build_files, oracle_range_info


def _row(buf, ri, deferred=False):
    o = O.readall(buf, ri)
    return shard.range_row((o["status"], o["fail_record"], o["n_records"], o["last_crc"]),
                           oracle_range_info(buf, ri), ri, deferred)


def _join(parts, rig):
    rows, blobs = zip(*[_row(b, ri) for b, ri in parts])
    return shard.join_rows(list(rows), list(blobs), rig)


def _whole(buf, rig):
    o = O.readall(buf, rig)
    return o["status"], (o["fail_record"] if o["status"] not in (O.OK, O.ERR_INDEX_NOT_FOUND) else -1), o["n_records"]


def _resolved(files, k_split, rig):
    """join the ranges, reading ranges k.. joined while the join asks"""
    parts = [(b"".join(b for b, _ in files[:k_split]), rig), (b"".join(b for b, _ in files[k_split:]),
                                                              max(rig, files[k_split][1]))]
    for _ in range(3):
        v = _join(parts, rig)
        if v[3] < 0:
            return v[:3]
        k = v[3]
        parts = parts[:k] + [(b"".join(b for b, _ in parts[k:]), parts[k][1])] + [(b"", 0)] * (len(parts) - k - 1)
    raise AssertionError("no final verdict")


def test_join_by_file_clean_and_dangling_prefix():
    rng = random.Random(5)
    for dangling in (False, True):
        files = [(bytes(b), i) for b, i in build_files(rng, 4)]
        if dangling:   # file 1 ends with a bare length prefix: alone it reads as io.EOF
            files[1] = (files[1][0] + struct.pack("<q", 40), files[1][1])
        allb = b"".join(b for b, _ in files)
        assert _resolved(files, 2, 0) == _whole(allb, 0)
        if dangling:   # the range alone is clean but short of its end: the join reads it joined
            parts = [(b"".join(b for b, _ in files[:2]), 0), (b"".join(b for b, _ in files[2:]), files[2][1])]
            assert _join(parts, 0)[3] == 0


def _deferred_row(status, pre, stored, u0, dlen):
    info = dict(n_frames=1, first_crc=-1, md_first_frame=-1, md_value_frame=-1, first_entry_frame=0,
                last_entry_frame=0, last_op_frame=0, first_type=2, first_entry_index=5, min_entry_index=5,
                last_entry_index=5, last_op_index=5, first_dlen=dlen, first_stored_crc=stored, first_u0=u0,
                first_pre_crc=pre, end_off=100, n_bytes=100)
    return shard.range_row((status, 0, 0, 0), info, 5, deferred=True)


def test_join_deferred_frame0_failure_classes():
    """a range's frame 0 failing on its own read.  A failure
    decoder.decode reports before its CRC check (framing, Record.Unmarshal:
    first_pre_crc) is the verdict; one that comes after it (Entry / HardState
    Unmarshal, e.g. PANIC_BOUNDS on a negative Entry.Data length) loses to the
    deferred CRC mismatch -- walpb.ErrCRCMismatch at the range's frame 0."""
    wal = O.WalEncoder(0)
    wal.save_crc(0)
    wal.encode(1, b"md")
    for i in range(1, 5):
        wal.save_entry(0, 1, i, bytes(range(i * 10)))
    head = wal.getvalue()
    r0 = _row(head, 1)
    n0 = O.readall(head, 1)["n_records"]
    data = b"not the data the stored CRC covers"
    u0 = O.crc32_update(0, data)
    for pre, want in ((1, O.PANIC_BOUNDS), (0, O.ERR_RECORD_CRC)):
        r1 = _deferred_row(O.PANIC_BOUNDS, pre, 0x1234, u0, len(data))
        v = shard.join_rows([r0[0], r1[0]], [r0[1], r1[1]], 1)
        assert v[:3] == (want, n0, n0), (pre, v)
    # the deferred check holding: the range's own failure stands
    running = O.readall(head, 1)["last_crc"]
    good = O.crc32_update(running, data)
    r1 = _deferred_row(O.PANIC_BOUNDS, 0, good, u0, len(data))
    assert shard.join_rows([r0[0], r1[0]], [r0[1], r1[1]], 1)[:3] == (O.PANIC_BOUNDS, n0, n0)


def _state_only_last_file(rng, nfiles=3):
    """wal.Create + Save + Cut, then a last file holding only crcType,
    metadata and a HardState with unknown fields (Save(st, nil) after the
    Cut): its name index is the next entry Index, so its own ReadAll (w.ri =
    that index, no entry op) ends in ErrIndexNotFound and keeps no side list."""
    files = [(bytes(b), i) for b, i in build_files(rng, nfiles)]
    allb = b"".join(b for b, _ in files)
    o = O.readall(allb, 0)
    e = O.WalEncoder(o["last_crc"])
    e.save_crc(o["last_crc"])
    e.encode(1, b"metadata")
    e.encode(3, O.hardstate_marshal(1, 1, o["enti"]) + bytes([0x20, 0x05]))
    return files + [(e.getvalue(), o["enti"] + 1)]


def test_join_state_unrec_in_entryless_last_file():
    """the last range holding the HardState (with
    XXX_unrecognized) has no entry op, so its own read is ErrIndexNotFound
    and the join must read joined -- from an EARLIER range whose read ended
    OK, so that the re-read settles (reading from the state range again gave
    the same rows forever and EWAL_E_INVAL).  By file, w.ri >= 1, 2 and 3
    ranges: the resolved verdict is the whole ReadAll's."""
    rng = random.Random(41)
    files = _state_only_last_file(rng)
    allb = b"".join(b for b, _ in files)
    for rig in (1, 3):
        whole = O.readall(allb, rig)
        assert whole["status"] == O.OK and whole["state"]["unrec"] == bytes([0x20, 0x05])
        assert _resolved(files, len(files) - 1, rig) == _whole(allb, rig)
        # three ranges: files [0, 1), [1, 3), [3]
        parts = [(files[0][0], rig), (files[1][0] + files[2][0], max(rig, files[1][1])),
                 (files[3][0], max(rig, files[3][1]))]
        v = _join(parts, rig)
        assert v[0] == O.OK and v[3] == 1, v   # the state range is 2: re-read from range 1 (its read ended OK)
        assert _row(parts[2][0], parts[2][1])[0].status == O.ERR_INDEX_NOT_FOUND
        joined = parts[:1] + [(parts[1][0] + parts[2][0], parts[1][1]), (b"", 0)]
        v2 = _join(joined, rig)
        assert v2[:3] == _whole(allb, rig) and v2[3] == -1, v2
