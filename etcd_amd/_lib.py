"""ctypes binding of libewal.so (include/ewal.h).

The shared library is built in-tree by etcd_amd/build.sh (hipcc, gfx950).
There is no CPU fallback: if the library is missing this module raises at
import, and every compute call on a machine without a GPU returns
EWAL_E_NODEVICE, which the wrappers raise as NoDeviceError.
"""
import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# EWAL_LIB_PATH: an alternative build of the same library (A/B timing runs
# in tools/ only); the default is the in-tree build.
LIB_PATH = os.environ.get("EWAL_LIB_PATH") or os.path.join(_HERE, "libewal.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "ewal.h")

if not os.path.exists(LIB_PATH):
    raise ImportError("etcd_amd: %s is missing -- run etcd_amd/build.sh (hipcc --offload-arch=gfx950)" % LIB_PATH)

# One HIP runtime per process: torch ships its own libamdhip64 (SONAME
# libamdhip64.so.7).  Loaded first, our DT_NEEDED libamdhip64.so.7 resolves
# to it; loaded after us, torch would map a second runtime and one of the two
# sees no device (measured on the MI355X box).  So torch, when importable,
# is imported before libewal.so is mapped.
if os.environ.get("EWAL_NO_TORCH") != "1":
    try:
        import torch  # noqa: F401
    except Exception:
        pass

lib = C.CDLL(LIB_PATH)

# ---- status codes (include/ewal.h) --------------------------------------
OK = 0
EOF = 1
ERR_UNEXPECTED_EOF = 2
ERR_RECORD_CRC = 3
ERR_WAL_CRC = 4
ERR_METADATA_CONFLICT = 5
ERR_INDEX_NOT_FOUND = 6
ERR_WRONG_TYPE = 7
ERR_UNEXPECTED_TYPE = 8
ERR_FILE_NOT_FOUND = 9
ERR_SNAP_CRC = 10
ERR_NO_SNAPSHOT = 11
PANIC_NEG_LENGTH = 32
PANIC_BOUNDS = 33
PANIC_ENTRY = 34
PANIC_STATE = 35
PANIC_INDEX_GAP = 36
NONTERMINATING = 37
UNSUPPORTED_ENCODING = 48
E_HIP, E_INVAL, E_NOMEM, E_NODEVICE, E_TIMEOUT, E_IO = -1, -2, -3, -4, -5, -6

FLAG_SHARD_FALLBACK = 1   # ewal_readall_batch_device verified this shard on its own
FLAG_METADATA_SPLIT = 2   # metadata_off / _len index the split bytes (ewal_copy_split_bytes)
FLAG_FAST_PATH = 4        # the fused frame pass decided this result (diagnostics)
OPT_GENERAL_PATH = 1      # ewal_ctx_set_options: every ReadAll on the general path
OPT_OVERLAP = 2           # ewal_ctx_set_options: the overlapped stream / frame pipeline (opt-in)
OPT_VH_ON = 4             # ewal_ctx_set_options: the frame pass's 128-B prefixes forced on (default: record-dense WALs)
OPT_VH_OFF = 8            # ... forced off
RANGE_DEFER_FIRST = 1     # ewal_readall_range_device: frame 0's CRC check is the caller's

CASTAGNOLI, IEEE, KOOPMAN = 0x82F63B78, 0xEDB88320, 0xEB31D82E


class MessageDesc(C.Structure):   # emsg_message
    _fields_ = [("status", C.c_int32), ("reject", C.c_int32), ("type", C.c_uint64), ("to", C.c_uint64),
                ("from_", C.c_uint64), ("term", C.c_uint64), ("log_term", C.c_uint64), ("index", C.c_uint64),
                ("commit", C.c_uint64), ("ents_first", C.c_uint64), ("n_ents", C.c_uint64),
                ("snap_index", C.c_uint64), ("snap_term", C.c_uint64), ("snap_data_off", C.c_int64),
                ("snap_data_len", C.c_int64), ("snap_n_nodes", C.c_uint64), ("snap_n_removed", C.c_uint64),
                ("unrec_len", C.c_int64), ("segs_first", C.c_uint64), ("n_segs", C.c_uint64)]


class SegmentDesc(C.Structure):   # emsg_segment
    _fields_ = [("kind", C.c_int32), ("pad", C.c_int32), ("ent", C.c_int64), ("off", C.c_uint64), ("len", C.c_uint64)]


SNAP_FIELD_DATA, SNAP_FIELD_UNREC, SNAP_FIELD_NODES, SNAP_FIELD_REMOVED = range(4)
SEG_UNREC, SEG_ENTRY_UNREC, SEG_ENTRY_DATA, SEG_SNAP_UNREC, SEG_SNAP_DATA, SEG_SNAP_NODE, SEG_SNAP_REMOVED = range(7)


class Result(C.Structure):
    _fields_ = [("status", C.c_int32), ("flags", C.c_int32), ("detail", C.c_int64), ("fail_record", C.c_int64),
                ("fail_offset", C.c_int64), ("n_records", C.c_int64), ("last_crc", C.c_uint32),
                ("n_unrec", C.c_uint32), ("enti", C.c_uint64), ("metadata_off", C.c_int64),
                ("metadata_len", C.c_int64), ("has_state", C.c_int32), ("n_slow", C.c_int32),
                ("state_term", C.c_uint64), ("state_vote", C.c_uint64), ("state_commit", C.c_uint64),
                ("n_ents", C.c_int64), ("n_candidates", C.c_int64), ("n_runs", C.c_int64), ("device_ms", C.c_double),
                ("stream_ms", C.c_double), ("post_ms", C.c_double), ("frames_ms", C.c_double)]


class EntryDesc(C.Structure):
    _fields_ = [("term", C.c_uint64), ("index", C.c_uint64), ("data_off", C.c_uint64), ("data_len", C.c_uint64),
                ("type", C.c_int32), ("data_nil", C.c_int32)]


class SaveRec(C.Structure):      # ewal_save_rec
    _fields_ = [("kind", C.c_int32), ("etype", C.c_int32), ("a", C.c_uint64), ("b", C.c_uint64), ("c", C.c_uint64),
                ("data_off", C.c_uint64), ("data_len", C.c_uint64), ("data_nil", C.c_int32), ("pad", C.c_int32)]


SAVE_ENTRY, SAVE_STATE, SAVE_CUT = 2, 3, 4


class UnrecDesc(C.Structure):    # ewal_unrec
    _fields_ = [("ent", C.c_int64), ("off", C.c_uint64), ("len", C.c_uint64)]


class RecordDesc(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("data_off", C.c_uint64), ("data_len", C.c_uint64), ("type", C.c_int64),
                ("crc", C.c_uint32), ("chained_crc", C.c_uint32)]


class RangeInfo(C.Structure):   # ewal_range_info
    _fields_ = [("n_frames", C.c_int64), ("first_crc", C.c_int64), ("md_first_frame", C.c_int64),
                ("md_first_off", C.c_int64), ("md_first_len", C.c_int64), ("md_value_frame", C.c_int64),
                ("md_value_off", C.c_int64), ("md_value_len", C.c_int64), ("first_entry_frame", C.c_int64),
                ("last_entry_frame", C.c_int64), ("first_entry_index", C.c_uint64),
                ("min_entry_index", C.c_uint64), ("last_entry_index", C.c_uint64), ("last_op_frame", C.c_int64),
                ("last_op_index", C.c_uint64), ("md_split", C.c_int32), ("first_pre_crc", C.c_int32),
                ("first_type", C.c_int64), ("first_dlen", C.c_uint64), ("first_stored_crc", C.c_uint32),
                ("first_u0", C.c_uint32), ("end_off", C.c_uint64), ("n_bytes", C.c_uint64),
                ("state_frame", C.c_int64), ("state_term", C.c_uint64), ("state_vote", C.c_uint64),
                ("state_commit", C.c_uint64), ("state_unrec", C.c_int32), ("pad2", C.c_int32)]


class RangeRow(C.Structure):    # ewal_range_row
    _fields_ = [("status", C.c_int32), ("deferred", C.c_int32), ("fail_record", C.c_int64),
                ("n_records", C.c_int64), ("ri", C.c_uint64), ("last_crc", C.c_uint32), ("pad", C.c_uint32),
                ("detail", C.c_int64), ("info", RangeInfo)]


class SplitResult(C.Structure):  # ewal_split_result
    _fields_ = [("status", C.c_int32), ("resplit", C.c_int32), ("fail_record", C.c_int64),
                ("n_records", C.c_int64), ("detail", C.c_int64), ("last_crc", C.c_uint32), ("pad", C.c_uint32),
                ("enti", C.c_uint64), ("md_range", C.c_int32), ("md_split", C.c_int32), ("md_off", C.c_int64),
                ("md_len", C.c_int64), ("md_blob_off", C.c_int64), ("state_range", C.c_int32), ("pad2", C.c_int32),
                ("state_term", C.c_uint64), ("state_vote", C.c_uint64), ("state_commit", C.c_uint64),
                ("n_ents", C.c_int64)]


class SnapshotDesc(C.Structure):
    _fields_ = [("index", C.c_uint64), ("term", C.c_uint64), ("data_off", C.c_uint64), ("data_len", C.c_uint64),
                ("n_nodes", C.c_int64), ("n_removed", C.c_int64), ("nodes", C.c_uint64 * 64),
                ("removed", C.c_uint64 * 64)]


vp = C.c_void_p
u8p = C.POINTER(C.c_uint8)
_SIGS = {
    "ewal_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "ewal_ctx_destroy": (None, [vp]),
    "ewal_ctx_set_stream": (C.c_int, [vp, vp]),
    "ewal_ctx_reserve": (C.c_int, [vp, C.c_uint64, C.c_uint32]),
    "ewal_ctx_set_options": (C.c_int, [vp, C.c_uint32]),
    "ewal_wal_size": (C.c_uint64, [vp]),
    "ewal_status_string": (C.c_char_p, [C.c_int]),
    "ewal_last_device_ms": (C.c_float, [vp]),
    "ewal_device_count": (C.c_int, []),
    "ewal_readall_device": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.POINTER(Result)]),
    "ewal_device_alloc": (C.c_int, [vp, C.c_uint64, C.POINTER(vp)]),
    "ewal_device_free": (C.c_int, [vp, vp]),
    "ewal_upload": (C.c_int, [vp, vp, vp, C.c_uint64]),
    "ewal_download": (C.c_int, [vp, vp, vp, C.c_uint64]),
    "ewal_stage_to_device": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(vp)]),
    "ewal_readall_host": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.POINTER(Result)]),
    "ewal_copy_entries": (C.c_int64, [vp, C.POINTER(EntryDesc), C.c_int64]),
    "ewal_last_stream_ms": (C.c_float, [vp]),
    "ewal_readall_batch_device": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                            C.POINTER(Result)]),
    "emsg_decode_batch_device": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                           C.c_uint32, C.POINTER(MessageDesc), C.POINTER(C.c_uint64)]),
    "emsg_copy_entries": (C.c_int64, [vp, C.c_uint64, C.POINTER(EntryDesc), C.c_int64]),
    "emsg_copy_segments": (C.c_int64, [vp, C.c_uint64, C.POINTER(SegmentDesc), C.c_int64]),
    "esnap_copy_field": (C.c_int64, [vp, C.c_uint32, C.c_int32, vp, C.c_int64]),
    "ewal_batch_copy_entries": (C.c_int64, [vp, C.c_uint64, C.POINTER(EntryDesc), C.c_int64]),
    "ewal_copy_records": (C.c_int64, [vp, C.POINTER(RecordDesc), C.c_int64]),
    "ewal_batch_copy_unrec": (C.c_int64, [vp, C.c_uint64, C.POINTER(UnrecDesc), C.c_int64]),
    "ewal_batch_copy_unrec_bytes": (C.c_int64, [vp, C.c_uint64, vp, C.c_int64]),
    "ewal_copy_range_info": (C.c_int, [vp, C.POINTER(RangeInfo)]),
    "ewal_split_verdict": (C.c_int, [C.POINTER(RangeRow), C.c_uint64, C.c_uint64, vp, C.c_uint64,
                                     C.POINTER(SplitResult)]),
    "ewal_readall_multi": (C.c_int, [C.POINTER(vp), C.c_uint32, vp, C.c_uint64, C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64), C.c_uint32, C.c_uint64, C.POINTER(SplitResult),
                                     C.POINTER(C.c_uint32)]),
    "ewal_split_ents_layout": (C.c_int64, [C.POINTER(RangeRow), C.c_uint64, C.c_uint64, C.POINTER(C.c_int64),
                                           C.POINTER(C.c_int64)]),
    "ewal_range_probe_aligned": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                           C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "ewal_multi_create": (C.c_int, [C.POINTER(vp), C.c_uint32, C.POINTER(vp)]),
    "ewal_multi_destroy": (None, [vp]),
    "ewal_multi_readall": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32,
                                     C.c_uint64, C.POINTER(SplitResult)]),
    "ewal_multi_readall_device": (C.c_int, [vp, C.POINTER(vp), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                            C.POINTER(C.c_uint32), C.c_uint64, C.POINTER(SplitResult)]),
    "ewal_multi_plan_device": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint64)]),
    "ewal_multi_copy_entries": (C.c_int64, [vp, C.POINTER(EntryDesc), C.c_int64]),
    "ewal_multi_copy_metadata": (C.c_int64, [vp, vp, C.c_int64]),
    "ewal_multi_copy_split_bytes": (C.c_int64, [vp, vp, C.c_int64]),
    "ewal_multi_copy_unrec": (C.c_int64, [vp, C.POINTER(UnrecDesc), C.c_int64]),
    "ewal_multi_copy_unrec_bytes": (C.c_int64, [vp, vp, C.c_int64]),
    "ewal_multi_copy_rows": (C.c_int, [vp, C.POINTER(RangeRow), C.POINTER(C.c_uint64), C.c_uint32]),
    "ewal_multi_timing": (C.c_int, [vp, C.POINTER(C.c_double)]),
    "ewal_copy_unrec": (C.c_int64, [vp, C.POINTER(UnrecDesc), C.c_int64]),
    "ewal_copy_unrec_bytes": (C.c_int64, [vp, vp, C.c_int64]),
    "ewal_copy_split_bytes": (C.c_int64, [vp, vp, C.c_int64]),
    "ewal_readall_range_device": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(Result)]),
    "ewal_range_probe": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_int64),
                                   C.POINTER(C.c_int64)]),
    "ewal_batch_copy_split_bytes": (C.c_int64, [vp, C.c_uint64, vp, C.c_int64]),
    "ewal_open_at_index": (C.c_int, [C.c_char_p, C.c_uint64, C.POINTER(vp)]),
    "ewal_wal_readall": (C.c_int, [vp, vp, C.POINTER(Result)]),
    "ewal_wal_bytes": (u8p, [vp, C.POINTER(C.c_uint64)]),
    "ewal_wal_seq": (C.c_uint64, [vp]),
    "ewal_wal_prefetch": (C.c_int, [vp]),
    "ewal_wal_close": (None, [vp]),
    "ewal_parse_wal_name": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "ewal_search_index": (C.c_int64, [C.POINTER(C.c_char_p), C.c_uint64, C.c_uint64]),
    "ewal_is_valid_seq": (C.c_int, [C.POINTER(C.c_char_p), C.c_uint64]),
    "ewal_wal_name": (None, [C.c_uint64, C.c_uint64, C.c_char_p]),
    "esnap_names": (C.c_int64, [C.c_char_p, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "ewal_create": (C.c_int, [C.c_char_p, C.c_char_p, C.c_uint64, C.c_int, C.POINTER(vp)]),
    "ewal_writer_save_entry": (C.c_int, [vp, C.c_int32, C.c_uint64, C.c_uint64, C.c_char_p, C.c_uint64]),
    "ewal_writer_save_state": (C.c_int, [vp, C.c_uint64, C.c_uint64, C.c_uint64]),
    "ewal_writer_cut": (C.c_int, [vp]),
    "ewal_writer_sync": (C.c_int, [vp]),
    "ewal_writer_close": (None, [vp]),
    "ewal_encoder_new": (vp, [C.c_uint32, C.c_uint64]),
    "ewal_encoder_encode": (C.c_int, [vp, C.c_int64, C.c_char_p, C.c_uint64, C.c_int]),
    "ewal_encoder_save_entry": (C.c_int, [vp, C.c_int32, C.c_uint64, C.c_uint64, C.c_char_p, C.c_uint64]),
    "ewal_encoder_save_state": (C.c_int, [vp, C.c_uint64, C.c_uint64, C.c_uint64]),
    "ewal_encoder_bytes": (u8p, [vp, C.POINTER(C.c_uint64)]),
    "ewal_encoder_crc": (C.c_uint32, [vp]),
    "ewal_encoder_free": (None, [vp]),
    "ewal_encode_entries_device": (C.c_int, [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, vp, C.c_uint64,
                                             C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    "ewal_save_device": (C.c_int, [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, vp, C.c_uint64,
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), vp]),
    "ewal_crc32_update_device": (C.c_int, [vp, C.c_uint32, C.c_uint32, vp, C.c_uint64, C.POINTER(C.c_uint32)]),
    "ewal_crc32_update_host": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_char_p, C.c_uint64]),
    "ewal_crc32_combine": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64]),
    "esnap_verify_packed": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32,
                                      C.c_uint32, C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_uint32)]),
    "esnap_copy_snapshot": (C.c_int, [vp, C.c_uint32, C.POINTER(SnapshotDesc)]),
    "esnap_load_dir": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.POINTER(SnapshotDesc), C.POINTER(C.c_char_p)]),
    "ecommit_batch_device": (C.c_int, [vp, C.c_uint64, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.POINTER(C.c_double)]),
    "ecommit_batch_rec_device": (C.c_int, [vp, C.c_uint64, vp, vp, vp, vp, vp, vp, C.POINTER(C.c_double)]),
}
for _name, (_res, _args) in _SIGS.items():
    if os.environ.get("EWAL_LIB_PATH") and not hasattr(lib, _name):
        continue   # an older A/B build (tools/ab_run.py) without a newer entry point
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


_synth = None


def synth_lib():
    """libewal_synth.so (include/ewal_synth.h): the synthetic-WAL generator of
    bench.py and the tests -- plumbing, not part of the product library."""
    global _synth
    if _synth is None:
        _synth = C.CDLL(os.path.join(_HERE, "libewal_synth.so"))
        _synth.ewal_synth_wal.restype = C.c_int64
        _synth.ewal_synth_wal.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int64, vp, C.c_uint64,
                                          C.POINTER(C.c_int64)]
        _synth.ewal_synth_wal_ex.restype = C.c_int64
        _synth.ewal_synth_wal_ex.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int64, C.c_uint32,
                                             vp, C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_uint64)]
    return _synth


def header_symbols(path=HEADER):
    """Every function declared in include/ewal.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(e(?:wal|snap|commit)_[a-z0-9_]+)\s*\(", txt)))


def status_string(st):
    return lib.ewal_status_string(st).decode()


class EwalError(Exception):
    """An EWAL_* status: the Go sentinel or panic class of the reference."""

    def __init__(self, status, detail=0, record=-1, offset=-1):
        self.status, self.detail, self.record, self.offset = status, detail, record, offset
        msg = status_string(status)
        if status == ERR_UNEXPECTED_TYPE:
            msg = "unexpected block type %d" % detail
        super().__init__(msg)


class NoDeviceError(EwalError):
    pass


class GoPanic(EwalError):
    """The reference panics here (make/slice bounds/mustUnmarshal*)."""


def check(st, detail=0, record=-1, offset=-1):
    if st == OK:
        return
    if st == E_NODEVICE:
        raise NoDeviceError(st)
    if 32 <= st <= 37:
        raise GoPanic(st, detail, record, offset)
    raise EwalError(st, detail, record, offset)
