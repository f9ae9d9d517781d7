/*
 * ewal.h -- C ABI of the MI355X-native etcd WAL replay-and-verify engine.
 *
 * Drop-in boundary for the reference's (mzsanford/etcd v0.5.0-alpha) hot
 * path.  Each entry point names the Go interface it replaces (file:line,
 * relative to the reference root).  A cgo shim binds these
 * with plain pointers and sizes; no HIP or torch types cross the boundary
 * except opaque handles and device pointers given as `const void *`.
 *
 * Ownership: the caller owns every buffer passed in; the library owns its
 * device workspace and stream inside an ewal_ctx.  Threading: one ctx per
 * host thread; calls are blocking.  Errors: a negative return is an
 * infrastructure failure (HIP); a non-negative return is an EWAL_* status
 * that maps 1:1 onto the reference's sentinel errors and panic classes.
 * There is no CPU fallback: without a usable GPU every compute entry point
 * returns EWAL_E_NODEVICE.
 */
#ifndef EWAL_H
#define EWAL_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (same numbering as oracle/ewal_oracle.h) ------------ */
enum {
  EWAL_OK = 0,
  EWAL_EOF = 1,                    /* io.EOF: clean end (internal only) */
  EWAL_ERR_UNEXPECTED_EOF = 2,     /* io.ErrUnexpectedEOF */
  EWAL_ERR_RECORD_CRC = 3,         /* walpb.ErrCRCMismatch   wal/walpb/record.go:22 */
  EWAL_ERR_WAL_CRC = 4,            /* wal.ErrCRCMismatch     wal/wal.go:48 */
  EWAL_ERR_METADATA_CONFLICT = 5,  /* wal.ErrMetadataConflict wal/wal.go:45 */
  EWAL_ERR_INDEX_NOT_FOUND = 6,    /* wal.ErrIndexNotFound   wal/wal.go:47 */
  EWAL_ERR_WRONG_TYPE = 7,         /* proto.ErrWrongType */
  EWAL_ERR_UNEXPECTED_TYPE = 8,    /* "unexpected block type %d" wal/wal.go:194; detail = type */
  EWAL_ERR_FILE_NOT_FOUND = 9,     /* wal.ErrFileNotFound    wal/wal.go:46 */
  EWAL_ERR_SNAP_CRC = 10,          /* snap.ErrCRCMismatch    snap/snapshotter.go:25 */
  EWAL_ERR_NO_SNAPSHOT = 11,       /* snap.ErrNoSnapshot     snap/snapshotter.go:24 */
  EWAL_PANIC_NEG_LENGTH = 32,      /* make([]byte, l<0)      wal/decoder.go:34 */
  EWAL_PANIC_BOUNDS = 33,          /* runtime bounds panic in Unmarshal/Skip */
  EWAL_PANIC_ENTRY = 34,           /* mustUnmarshalEntry     wal/decoder.go:61-69 */
  EWAL_PANIC_STATE = 35,           /* mustUnmarshalState     wal/decoder.go:71-77 */
  EWAL_PANIC_INDEX_GAP = 36,       /* ents[:e.Index-ri] past len wal/wal.go:173 */
  EWAL_NONTERMINATING = 37,        /* the reference never returns */
  EWAL_UNSUPPORTED_ENCODING = 48,  /* protobuf groups nested deeper than the device
                                      walker's stack; reported, never guessed */
  /* infrastructure (negative) */
  EWAL_E_HIP = -1,
  EWAL_E_INVAL = -2,
  EWAL_E_NOMEM = -3,
  EWAL_E_NODEVICE = -4,
  EWAL_E_TIMEOUT = -5,
  EWAL_E_IO = -6
};

/* Record types, wal/wal.go:34-39 */
enum { EWAL_METADATA = 1, EWAL_ENTRY = 2, EWAL_STATE = 3, EWAL_CRC = 4 };

typedef struct ewal_ctx ewal_ctx;

/* Result of (*WAL).ReadAll, wal/wal.go:164-216.  On error the reference
 * returns (nil, HardState{}, nil, err): only status/detail/fail_* and
 * n_records are meaningful then. */
typedef struct ewal_result {
  int32_t status;          /* EWAL_OK or an EWAL_ERR_/EWAL_PANIC_ class */
  int32_t flags;
  int64_t detail;          /* unexpected block type value; gap index */
  int64_t fail_record;     /* ordinal of the frame that failed, -1 if none */
  int64_t fail_offset;     /* byte offset of that frame in the stream, -1 */
  int64_t n_records;       /* frames decoded before the end / failure */
  uint32_t last_crc;       /* decoder.lastCRC() -> seeds the encoder, wal/wal.go:213 (set with
                              ErrIndexNotFound too: a split WAL's next range starts from it) */
  uint32_t n_unrec;        /* ents / HardState carrying XXX_unrecognized: ewal_copy_unrec */
  uint64_t enti;           /* w.enti: Index of the last entry record */
  int64_t metadata_off;    /* metadata []byte as (offset,len) into the stream; -1 == nil */
  int64_t metadata_len;
  int32_t has_state;       /* 0 -> HardState{} */
  int32_t n_slow;          /* diagnostics: frames decoded by the general (non-canonical) walker */
  uint64_t state_term, state_vote, state_commit;
  int64_t n_ents;          /* len(ents); fetch with ewal_copy_entries */
  int64_t n_candidates;    /* diagnostics: frame-start candidates found */
  int64_t n_runs;          /* diagnostics: chain runs in the framing pass */
  double device_ms;        /* device time of the pipeline (HIP events) */
  double stream_ms;        /* device time of the k_stream HBM pass alone */
  double post_ms;          /* device time from the end of the stream pass to the end of the pipeline: the part
                              of device_ms the stream pass does not hide (diagnostics) */
  double frames_ms;        /* device time of the frame pass kernel k_frames, when it ran as one launch after the
                              stream pass (0 in the overlapped pipeline, where post_ms is its exposed part) */
} ewal_result;

/* raftpb.Entry, raft/raftpb/raft.pb.go:100-106.  Data is a zero-copy
 * (offset,len) view of the stream; data_nil mirrors Go's nil slice.
 * data_nil == 2: Data is instead the range [data_off, data_off + data_len) of
 * the split bytes (ewal_copy_split_bytes / ewal_batch_copy_split_bytes) -- the
 * concatenation Go's append builds when the Entry's Data, or the Record.Data
 * holding the Entry, is repeated with several non-empty segments
 * (raft.pb.go:254, wal/walpb/record.pb.go:112; etcd's encoder never writes
 * that, a crafted WAL can). */
typedef struct ewal_entry {
  uint64_t term;
  uint64_t index;
  uint64_t data_off;
  uint64_t data_len;
  int32_t type;
  int32_t data_nil;
} ewal_entry;

/* XXX_unrecognized of a returned Entry / the HardState (raft.pb.go:100-106,
 * 143-148: the unknown fields Unmarshal appended, raft.pb.go:270), bytes at
 * [off, off+len) of the side buffer (ewal_copy_unrec_bytes).  Entries and a
 * HardState not listed have a nil XXX_unrecognized. */
typedef struct ewal_unrec {
  int64_t ent;             /* index into ents, or -1: the HardState */
  uint64_t off, len;
} ewal_unrec;

/* One decoded frame (walpb.Record + chain state), wal/walpb/record.pb.go:30-35 */
typedef struct ewal_record {
  uint64_t offset;         /* frame start (int64 length prefix) */
  uint64_t data_off;
  uint64_t data_len;
  int64_t type;
  uint32_t crc;            /* stored Record.Crc */
  uint32_t chained_crc;    /* decoder crc after this frame (== crc when it verified) */
} ewal_record;

/* ---- context ------------------------------------------------------------ */
int ewal_ctx_create(int device, ewal_ctx **out);
/* Releases every device resource of ctx.  Contract: destroy every ctx before
 * the process exits (a Go caller: before main returns / os.Exit).  The
 * library covers a ctx left alive with EWAL_OPT_OVERLAP: its two CU-masked
 * streams are destroyed by an atexit handler the library registers when it
 * creates them, before the HIP runtime's own teardown (round 6: such a ctx
 * crashed in __cxa_finalize at exit). */
void ewal_ctx_destroy(ewal_ctx *ctx);
/* Run on a caller-owned hipStream_t (NULL = the ctx's own stream).  The
 * ctx's own stream is a blocking stream: it is ordered with the legacy
 * default stream (stream 0, torch's default stream), so inputs written there
 * are complete before the ctx reads them.  A caller-owned non-blocking
 * stream gets no such ordering: the caller orders its own work on it. */
int ewal_ctx_set_stream(ewal_ctx *ctx, void *hip_stream);
/* Pre-size ctx's workspace for a ReadAll over up to wal_bytes and load the
 * device code, so that the first ReadAll (the one-shot restart,
 * etcdserver/server.go:153-156) allocates nothing.  A server calls it while
 * it reads the WAL files from disk: OpenAtIndex's directory listing gives
 * their total size first.  Optional: without it the first call sizes the
 * workspace itself. */
#define EWAL_RESERVE_HOST_STAGING 1u   /* also the HBM staging buffer of ewal_readall_host / ewal_wal_readall */
int ewal_ctx_reserve(ewal_ctx *ctx, uint64_t wal_bytes, uint32_t flags);
/* Path options of ctx (default 0: the fused frame pass first, the general
 * path when it cannot decide a WAL).  EWAL_OPT_GENERAL_PATH: every ReadAll
 * takes the general path (framing by candidate links, per-frame descriptors)
 * -- the same results, slower; for cross-checking the two paths.  No
 * environment variable changes the path. */
#define EWAL_OPT_GENERAL_PATH 1u
/* EWAL_OPT_OVERLAP: a single ReadAll of >= 512 MiB streams its bytes in four
 * chunks on 224 CUs (a CU-masked stream) while each finished chunk's frame
 * pass runs on the other 32 (a second CU-masked stream).  Off by default:
 * measured on MI355X it does not pay (profiles/r05/): the
 * stream pass loses speed faster than the frame pass gains CUs, and masks
 * of more than 32 CUs on the frame side slowed the stream side 2.4x.  A ctx
 * with this option owns two extra streams: destroy it before the process
 * exits (a live one is cleaned up at exit, see ewal_ctx_destroy). */
#define EWAL_OPT_OVERLAP 2u
/* Record-dense WALs (round 5): the stream pass also stores the lin of every
 * 256-B super-piece's first 128-B half, and the frame pass takes every frame
 * start's prefix from the nearest 128-B boundary instead of the nearest 256-B
 * one (half the tail bytes).  By default a ctx turns it on when its previous
 * single ReadAll had >= 4 frames per 4 KiB (average frame <= 1 KiB);
 * EWAL_OPT_VH_ON / EWAL_OPT_VH_OFF force it either way (the same results). */
#define EWAL_OPT_VH_ON 4u
#define EWAL_OPT_VH_OFF 8u
int ewal_ctx_set_options(ewal_ctx *ctx, uint32_t opts);
const char *ewal_status_string(int status);
/* Device time (ms) of the last pipeline call on this ctx (HIP events). */
float ewal_last_device_ms(ewal_ctx *ctx);
/* Device time (ms) of the last call's k_stream HBM pass (HIP events). */
float ewal_last_stream_ms(ewal_ctx *ctx);
int ewal_device_count(void);

/* ---- WAL replay/verify -------------------------------------------------- */
/* (*WAL).ReadAll over the concatenated bytes of OpenAtIndex's files
 * names[nameIndex:] (wal/wal.go:126-134, MultiReadCloser semantics), with
 * w.ri = ri.  d_buf is DEVICE memory, 16-byte aligned, len bytes. */
int ewal_readall_device(ewal_ctx *ctx, const void *d_buf, uint64_t len, uint64_t ri, ewal_result *out);
/* Batched ReadAll over n_shards independent WALs (one raft group's
 * names[nameIndex:] each) laid end to end in ONE device
 * buffer: shard s is the lens[s] bytes after shards 0..s-1; out[s] is exactly
 * ewal_readall_device's result for that shard alone with w.ri = ri[s]
 * (ordinals and offsets relative to the shard; stream_ms is the batch's
 * k_stream, device_ms the batch's pipeline plus any shard replayed alone).
 * One stream pass and one fused frame + check pass cover the batch; a shard
 * that pass cannot decide -- torn or corrupt framing, an index rewind, an
 * encoding the canonical parser declines, unknown fields -- is replayed alone
 * (flags |= EWAL_FLAG_SHARD_FALLBACK) while every other shard keeps the
 * batch's result.  Shards whose returned ents / HardState carry
 * XXX_unrecognized have n_unrec > 0 and a side list per shard
 * (ewal_batch_copy_unrec).  Returns 0 or a negative infrastructure error;
 * per-shard verdicts are in out[].  Replaces, per shard,
 * wal.OpenAtIndex(...).ReadAll() (wal/wal.go:108,164). */
#define EWAL_FLAG_SHARD_FALLBACK 1
/* ewal_result.flags: metadata_off / metadata_len index the split bytes (the
 * metadata record's Data repeated with several non-empty segments), not the
 * stream */
#define EWAL_FLAG_METADATA_SPLIT 2
/* ewal_result.flags (diagnostics): the fused frame pass decided this result
 * (no per-frame descriptors were built); absent: the general path did */
#define EWAL_FLAG_FAST_PATH 4
int ewal_readall_batch_device(ewal_ctx *ctx, const void *d_buf, uint64_t n_shards, const uint64_t *lens,
                              const uint64_t *ri, ewal_result *out);
/* After ewal_readall_batch_device: shard s's ents (Data offsets relative to
 * the shard).  Returns the number copied (<= cap) or a negative error. */
int64_t ewal_batch_copy_entries(ewal_ctx *ctx, uint64_t shard, ewal_entry *out, int64_t cap);
/* After ewal_readall_batch_device: shard s's XXX_unrecognized side list
 * (ewal_unrec, ent = index into that shard's ents or -1 for its HardState)
 * and the bytes it indexes.  Return the number copied (<= cap). */
int64_t ewal_batch_copy_unrec(ewal_ctx *ctx, uint64_t shard, ewal_unrec *out, int64_t cap);
int64_t ewal_batch_copy_unrec_bytes(ewal_ctx *ctx, uint64_t shard, uint8_t *out, int64_t cap);
/* Copy host bytes into ctx-owned device memory (16-B aligned; valid until
 * the next staging call on this ctx). */
int ewal_stage_to_device(ewal_ctx *ctx, const void *h_buf, uint64_t len, void **d_out);
/* Device memory owned by the caller through the library (for callers that
 * have no HIP runtime of their own, e.g. cgo): alloc/free/copy. */
int ewal_device_alloc(ewal_ctx *ctx, uint64_t len, void **d_out);
int ewal_device_free(ewal_ctx *ctx, void *d_buf);
int ewal_upload(ewal_ctx *ctx, void *d_dst, const void *h_src, uint64_t len);
int ewal_download(ewal_ctx *ctx, void *h_dst, const void *d_src, uint64_t len);
/* Same, from host memory: staged to the device first (PCIe-inclusive). */
int ewal_readall_host(ewal_ctx *ctx, const void *h_buf, uint64_t len, uint64_t ri, ewal_result *out);
/* After a successful readall: copy the ents / per-frame descriptors out.
 * Return the number copied (<= cap) or a negative error.  The descriptors
 * are rebuilt on demand from the ctx's stream-pass state and the ReadAll's
 * stream bytes: d_buf must still hold them (the same lifetime rule as the
 * ents' Data views), and any later compute call on the ctx (another ReadAll,
 * a batch, a CRC, snapshot or save call, a staging call that reuses the
 * staging buffer) makes ewal_copy_records return EWAL_E_INVAL. */
int64_t ewal_copy_entries(ewal_ctx *ctx, ewal_entry *out, int64_t cap);
int64_t ewal_copy_records(ewal_ctx *ctx, ewal_record *out, int64_t cap);
/* After a successful readall with n_unrec > 0: the side list (sorted by ent)
 * and its bytes. */
int64_t ewal_copy_unrec(ewal_ctx *ctx, ewal_unrec *out, int64_t cap);
int64_t ewal_copy_unrec_bytes(ewal_ctx *ctx, uint8_t *out, int64_t cap);
/* After a successful readall: the split bytes the data_nil == 2 ents and an
 * EWAL_FLAG_METADATA_SPLIT metadata index (gathered on the device).  Copies
 * min(cap, total) bytes; returns the total (0: none) or a negative error.
 * The batched form: shard s's (a shard with split fields is replayed alone). */
int64_t ewal_copy_split_bytes(ewal_ctx *ctx, uint8_t *out, int64_t cap);
int64_t ewal_batch_copy_split_bytes(ewal_ctx *ctx, uint64_t shard, uint8_t *out, int64_t cap);

/* What one rank's range of ONE WAL split by file contributes to the joined
 * verdict (etcd_amd/shard.py split_verdict applies ReadAll's
 * cross-file rules with it), from the last ReadAll on ctx over that range --
 * all frames of its chain, those after a failure included.  Frames are
 * ordinals in the range, offsets are into the range's stream (d_buf must
 * still hold it, as for ewal_copy_records).  The rules it serves:
 *   crc seam       wal/wal.go:184-192 (every file opens with crcType{running
 *                  CRC}, wal/wal.go:93,232-234)
 *   metadata       wal/wal.go:178-183
 *   ents / enti    wal/wal.go:170-174, 203-206 (the index-gap rule across the
 *                  range boundary, rewinds below the range's w.ri, and the
 *                  global ErrIndexNotFound) */
typedef struct ewal_range_info {
  int64_t n_frames;              /* frames on the chain */
  int64_t first_crc;             /* Crc of frame 0 when it is a crcType record, else -1 */
  int64_t md_first_frame;        /* the first metadataType frame, -1: none */
  int64_t md_first_off, md_first_len;   /* its Data; off -1 == nil */
  int64_t md_value_frame;        /* the first metadataType frame with non-nil Data (the value ReadAll keeps), -1 */
  int64_t md_value_off, md_value_len;
  int64_t first_entry_frame;     /* the first entryType frame, -1: none */
  int64_t last_entry_frame;
  uint64_t first_entry_index;    /* its Entry.Index */
  uint64_t min_entry_index;      /* the least Entry.Index of the range */
  uint64_t last_entry_index;     /* the last entry frame's Index (w.enti after the range) */
  int64_t last_op_frame;         /* the last entry frame with Index >= the ReadAll's ri (the last
                                    append to ents, wal/wal.go:171-173), -1: none */
  uint64_t last_op_index;
  int32_t md_split;              /* bit 0: md_first_off, bit 1: md_value_off index the split bytes
                                    (ewal_copy_split_bytes: a metadata Data in several segments) */
  int32_t first_pre_crc;         /* 1: frame 0 failed inside decoder.decode before its CRC check
                                    (framing, walpb.Record.Unmarshal, wal/decoder.go:30-41) -- that
                                    failure wins over the caller's deferred check; 0: it did not fail
                                    there (an Entry / HardState decode failure comes after the check) */
  /* frame 0 (EWAL_RANGE_DEFER_FIRST: the caller's CRC check) */
  int64_t first_type;            /* Record.Type, -1: no frame */
  uint64_t first_dlen;           /* len(Data) */
  uint32_t first_stored_crc;     /* Record.Crc */
  uint32_t first_u0;             /* crc32.Update(0, Castagnoli, Data) (the stored CRC for a crcType frame) */
  uint64_t end_off;              /* where the frame chain ended (decoder.decode's terminal): n_bytes when
                                    the range ended on a frame boundary */
  uint64_t n_bytes;              /* the range's length */
  /* the range's last stateType frame (ReadAll's `state = mustUnmarshalState`,
     wal/wal.go:176-177): the HardState the whole WAL returns when no later
     range holds one */
  int64_t state_frame;           /* -1: none */
  uint64_t state_term, state_vote, state_commit;
  int32_t state_unrec;           /* 1: that HardState carries XXX_unrecognized */
  int32_t pad2;
} ewal_range_info;
int ewal_copy_range_info(ewal_ctx *ctx, ewal_range_info *out);

/* ONE WAL split across ranks INSIDE a file: rank r takes the
 * bytes [c_r, c_{r+1}) of the stream, where c_r is the first frame-start
 * candidate at or after r * len / ranks (ewal_range_probe; c_0 = 0).  The
 * running CRC before a range's frame 0 is the previous range's, so with
 * EWAL_RANGE_DEFER_FIRST frame 0's CRC check (decoder.decode's Validate,
 * wal/decoder.go:42-46, or the crcType rule, wal/wal.go:184-192) is left to
 * the caller, who makes it with ewal_copy_range_info's first_* operands
 * (first_u0 = crc32.Update(0, Data), combined with the running CRC by
 * ewal_crc32_combine); every other rule is ReadAll's over the range with
 * w.ri = ri.  etcd_amd/shard.py split_verdict joins the ranges. */
#define EWAL_RANGE_DEFER_FIRST 1u
int ewal_readall_range_device(ewal_ctx *ctx, const void *d_buf, uint64_t len, uint64_t ri, uint32_t flags,
                              ewal_result *out);
/* The first frame-start candidate at or after `from` within `window` bytes of
 * a device stream of len bytes (*pos, -1: none), and the Index of the first
 * entry record on the frame chain from it within 64 frames (*first_entry_index,
 * -1: none) -- the range's w.ri candidate. */
int ewal_range_probe(ewal_ctx *ctx, const void *d_buf, uint64_t len, uint64_t from, uint64_t window, int64_t *pos,
                     int64_t *first_entry_index);
/* The same, taking only candidates at positions that are multiples of align
 * (a power of two): with 16 a range of a device-resident WAL starts on an
 * address every kernel can read without a copy (ewal_multi_plan_device). */
int ewal_range_probe_aligned(ewal_ctx *ctx, const void *d_buf, uint64_t len, uint64_t from, uint64_t window,
                             uint32_t align, int64_t *pos, int64_t *first_entry_index);

/* ---- ONE WAL over several ranges: ReadAll's verdict joined (host C++) ------
 * Range k of a WAL split into contiguous ranges (by file, or inside a file)
 * was read by ReadAll on its own (ewal_readall_device / _range_device with
 * w.ri = ri); its row carries that ReadAll's result and ewal_copy_range_info.
 * ewal_split_verdict applies ReadAll's cross-range rules in order, before
 * each range's own first failure (wal/wal.go:164-216):
 *   crc seam        a crcType frame 0 against the running CRC (wal/wal.go:184-192)
 *   deferred frame 0 (a range starting inside a file) Validate with the running
 *                   CRC, crc32.Update(running, Data) = ewal_crc32_combine(running,
 *                   first_u0, first_dlen) (wal/decoder.go:42-46)
 *   metadata        metadata != nil && !DeepEqual (wal/wal.go:178-183)
 *   ents            the range's first entry op against len(ents) carried over
 *                   (the index-gap panic, wal/wal.go:170-173); ErrIndexNotFound
 *                   over all ranges (wal/wal.go:203-206)
 * resplit = k >= 0: the verdict needs ranges k.. read as ONE range (a frame
 * cut short at range k's end, bytes range k left unconsumed, a rewind below a
 * range's w.ri): the caller reads them joined, marks the later rows empty
 * (n_bytes 0) and calls again.  md: the metadata bytes of every range in
 * order -- its first metadata frame's Data (when md_first_frame >= 0 and
 * md_first_off >= 0) then the value kept (md_value_frame >= 0). */
typedef struct ewal_range_row {
  int32_t status;                /* ReadAll's status over the range */
  int32_t deferred;              /* 1: read with EWAL_RANGE_DEFER_FIRST */
  int64_t fail_record;           /* the range's ordinal, -1 */
  int64_t n_records;
  uint64_t ri;                   /* the range's w.ri */
  uint32_t last_crc;             /* ReadAll's running CRC after the range */
  uint32_t pad;
  int64_t detail;                /* ReadAll's detail (block type, gap index) */
  ewal_range_info info;          /* ewal_copy_range_info of that ReadAll */
} ewal_range_row;
typedef struct ewal_split_result {
  int32_t status;
  int32_t resplit;               /* -1: final; k: read ranges k.. joined and call again */
  int64_t fail_record;           /* the global frame ordinal of the failure, -1 */
  int64_t n_records;             /* frames verified */
  int64_t detail;
  uint32_t last_crc;             /* decoder.lastCRC() after the WAL (EWAL_OK) */
  uint32_t pad;
  uint64_t enti;                 /* w.enti: the last entry's Index (EWAL_OK) */
  /* the rest of ReadAll's (metadata, state, ents) on EWAL_OK (wal/wal.go:206-215) */
  int32_t md_range;              /* the range whose metadata Data ReadAll returns, -1: nil */
  int32_t md_split;              /* 1: md_off indexes that range's split bytes, 0: its stream */
  int64_t md_off, md_len;        /* the Data inside that range */
  int64_t md_blob_off;           /* the same bytes inside the md blob given to ewal_split_verdict */
  int32_t state_range;           /* the range whose last HardState ReadAll returns, -1: HardState{} */
  int32_t pad2;
  uint64_t state_term, state_vote, state_commit;
  int64_t n_ents;                /* len(ents): ranges' ents stitched as ewal_split_ents_layout says */
} ewal_split_result;
int ewal_split_verdict(const ewal_range_row *rows, uint64_t n, uint64_t ri_global, const uint8_t *md, uint64_t md_len,
                       ewal_split_result *out);
/* Where each range's ents land in the joined ents of a final EWAL_OK verdict
 * (wal/wal.go:170-173, `ents = append(ents[:e.Index-w.ri], e)` carried across
 * the ranges): range k's ents (its own ReadAll's, with w.ri = rows[k].ri) are
 * joined ents [base[k], base[k] + count[k]), where base[k] = rows[k].ri - ri
 * and count[k] is cut where a later range's base overwrites them; ranges
 * without entry ops get count 0.  Returns len(ents) or a negative error. */
int64_t ewal_split_ents_layout(const ewal_range_row *rows, uint64_t n, uint64_t ri_global, int64_t *base,
                               int64_t *count);
/* ReadAll over ONE WAL (the bytes of names[nameIndex:], h_buf, len) split
 * across n_ctx contexts in one process -- one host thread per context, each
 * on its own device or sharing one: by file when file_off (n_files + 1
 * offsets, file_off[0] = 0, file_off[n_files] = len) and file_index (the
 * index in each file's name) are given, each range a run of whole files
 * with w.ri = max(ri, its first file's index); else inside the stream, range
 * r starting at the first frame-start candidate after r * len / n_ctx
 * (ewal_range_probe) with frame 0's check deferred.  The ranges' verdicts
 * are joined by ewal_split_verdict (re-reading ranges joined when it asks).
 * out->status etc. are exactly (*WAL).ReadAll's over the whole stream with
 * w.ri = ri; *n_resplit (nullable) counts the joined re-reads. */
int ewal_readall_multi(ewal_ctx *const *ctxs, uint32_t n_ctx, const void *h_buf, uint64_t len, const uint64_t *file_off,
                       const uint64_t *file_index, uint32_t n_files, uint64_t ri, ewal_split_result *out,
                       uint32_t *n_resplit);

/* ---- ONE WAL over several contexts: ReadAll's whole result ---------------
 * An ewal_multi drives n_ctx DISTINCT contexts (they may share a device; one
 * ctx is never used from two threads) and keeps, after each call, what
 * (*WAL).ReadAll returns over the whole stream (wal/wal.go:164-216, its
 * caller etcdserver/server.go:153-168): the verdict in ewal_split_result
 * (status, lastCRC, enti, the metadata's range and bytes, the HardState,
 * len(ents)) and, on EWAL_OK, the joined ents, metadata, split bytes and
 * XXX_unrecognized side list through the ewal_multi_copy_* calls -- which
 * read the ranges' ReadAll state left on each ctx: no other call may run on
 * those ctxs in between.  A ctx stays ordered with the legacy default stream
 * (ewal_ctx_set_stream); on a shared device a ctx's blocking stream also
 * waits for the others' null-stream allocations and copies, which is why the
 * host path stages into each ctx's reusable buffer instead of allocating. */
typedef struct ewal_multi ewal_multi;
int ewal_multi_create(ewal_ctx *const *ctxs, uint32_t n_ctx, ewal_multi **out);
void ewal_multi_destroy(ewal_multi *m);
/* From host bytes (each range staged into its ctx's staging buffer), split as
 * ewal_readall_multi says.  out->resplit is always -1 on return. */
int ewal_multi_readall(ewal_multi *m, const void *h_buf, uint64_t len, const uint64_t *file_off,
                       const uint64_t *file_index, uint32_t n_files, uint64_t ri, ewal_split_result *out);
/* Device-resident ranges: range r is the bytes [starts[r], starts[r + 1]) of
 * the stream, already in HBM at d_ranges[r] (16-B aligned) where ctx r reads
 * them, read with w.ri = ris[r] and flags[r] (EWAL_RANGE_DEFER_FIRST for a
 * range starting inside a file; flags NULL: every range but the first).  No
 * allocation, no host copy of the WAL.  A joined re-read the verdict asks for
 * runs on ctx k when ranges k.. form one contiguous device span; otherwise
 * out->resplit = k comes back and the caller reads ranges k.. joined itself. */
int ewal_multi_readall_device(ewal_multi *m, const void *const *d_ranges, const uint64_t *starts, const uint64_t *ris,
                              const uint32_t *flags, uint64_t ri, ewal_split_result *out);
/* Ranges of ONE device-resident stream d_buf[0, len) that every ctx of m can
 * read (the contexts on d_buf's device): starts[0..n_ctx] (range r opens at a
 * 16-B aligned frame-start candidate after r * len / n_ctx, found by
 * ewal_range_probe_aligned on ctx r) and each range's w.ri; then
 * d_ranges[r] = d_buf + starts[r] for ewal_multi_readall_device.  A range
 * whose 64 MiB probe window holds no aligned candidate is left empty
 * (starts[r] == starts[r + 1]: the range before reads on through it). */
int ewal_multi_plan_device(ewal_multi *m, const void *d_buf, uint64_t len, uint64_t ri, uint64_t *starts,
                           uint64_t *ris);
/* After a final EWAL_OK: len(ents) entries joined in order (Data offsets into
 * the whole stream, or into ewal_multi_copy_split_bytes for data_nil == 2),
 * the metadata Data (returns its length; 0 with md_range -1: nil), the
 * ranges' split bytes joined, the XXX_unrecognized side list (ent into the
 * joined ents, -1 the HardState; sorted) and its bytes.  Each returns the
 * total (entries, bytes) and copies min(cap, total). */
int64_t ewal_multi_copy_entries(ewal_multi *m, ewal_entry *out, int64_t cap);
int64_t ewal_multi_copy_metadata(ewal_multi *m, uint8_t *out, int64_t cap);
int64_t ewal_multi_copy_split_bytes(ewal_multi *m, uint8_t *out, int64_t cap);
int64_t ewal_multi_copy_unrec(ewal_multi *m, ewal_unrec *out, int64_t cap);
int64_t ewal_multi_copy_unrec_bytes(ewal_multi *m, uint8_t *out, int64_t cap);
/* The last call's ranges (rows and stream starts; returns n_ctx) and timing:
 * out4 = {wall ms of the call, the slowest range's device ms, host ms in the
 * join, joined re-reads}. */
int ewal_multi_copy_rows(ewal_multi *m, ewal_range_row *out, uint64_t *starts, uint32_t cap);
int ewal_multi_timing(ewal_multi *m, double *out4);

/* ---- directory-level API: wal.OpenAtIndex + ReadAll + writer ----------- */
typedef struct ewal_wal ewal_wal;
/* wal.OpenAtIndex(dirpath, index), wal/wal.go:108-159 (file selection:
 * wal/util.go:20-88): selects and opens names[nameIndex:]; their bytes are
 * read by ewal_wal_readall (pieces read by a few threads while the finished
 * ones are already copied to HBM) or on demand by ewal_wal_bytes. */
int ewal_open_at_index(const char *dirpath, uint64_t index, ewal_wal **out);
/* The file-name helpers OpenAtIndex uses (host-only), wal/util.go:20-88:
 * parseWalName (1 = parsed), searchIndex over sorted names (the index, -1
 * when none), isValidSeq (1 / 0), walName (out: 38 bytes). */
int ewal_parse_wal_name(const char *name, uint64_t *seq, uint64_t *index);
int64_t ewal_search_index(const char *const *names, uint64_t n, uint64_t index);
int ewal_is_valid_seq(const char *const *names, uint64_t n);
void ewal_wal_name(uint64_t seq, uint64_t index, char *out);
int ewal_wal_readall(ewal_wal *w, ewal_ctx *ctx, ewal_result *out);
/* total bytes of the opened files (size ewal_ctx_reserve before ReadAll) */
uint64_t ewal_wal_size(ewal_wal *w);
/* Start reading the opened files into host memory in the background (reader
 * threads, 64 MiB pieces) and return at once: a restarting server calls it
 * right after OpenAtIndex so the reads overlap its GPU context creation;
 * ewal_wal_readall then uploads the pieces already read and waits for the
 * rest.  Optional (ReadAll starts the reads itself). */
int ewal_wal_prefetch(ewal_wal *w);
const uint8_t *ewal_wal_bytes(ewal_wal *w, uint64_t *len);
uint64_t ewal_wal_seq(ewal_wal *w);
void ewal_wal_close(ewal_wal *w);

/* Write path (the on-disk format the hot path reads), wal/wal.go:72-100,
 * 219-292, wal/encoder.go:25-37.  Host C++; CRC via SSE4.2. */
typedef struct ewal_writer ewal_writer;
int ewal_create(const char *dirpath, const uint8_t *metadata, uint64_t mlen, int metadata_nil, ewal_writer **out);
int ewal_writer_save_entry(ewal_writer *w, int32_t type, uint64_t term, uint64_t index, const uint8_t *data, uint64_t n);
int ewal_writer_save_state(ewal_writer *w, uint64_t term, uint64_t vote, uint64_t commit);
int ewal_writer_cut(ewal_writer *w);
int ewal_writer_sync(ewal_writer *w);
void ewal_writer_close(ewal_writer *w);

/* In-memory encoder (encoder.encode over a growing buffer). */
typedef struct ewal_encoder ewal_encoder;
ewal_encoder *ewal_encoder_new(uint32_t prev_crc, uint64_t reserve);
int ewal_encoder_encode(ewal_encoder *e, int64_t type, const uint8_t *data, uint64_t n, int data_nil);
int ewal_encoder_save_entry(ewal_encoder *e, int32_t type, uint64_t term, uint64_t index, const uint8_t *data, uint64_t n);
int ewal_encoder_save_state(ewal_encoder *e, uint64_t term, uint64_t vote, uint64_t commit);
const uint8_t *ewal_encoder_bytes(ewal_encoder *e, uint64_t *len);
uint32_t ewal_encoder_crc(ewal_encoder *e);
void ewal_encoder_free(ewal_encoder *e);

/* ---- batched write path: (*WAL).SaveEntry / encoder.encode on the GPU ---- */
/* encoder.encode(&walpb.Record{Type: entryType, Data: pbutil.MustMarshal(e)})
 * for n entries in order (wal/wal.go:248-263, wal/encoder.go:25-37): the
 * frames, byte-identical to the reference's encoder, and the chained CRC
 * (c_i = crc32.Update(c_{i-1}, Castagnoli, Entry_i bytes), c_{-1} = prev_crc).
 * d_data: the entries' payloads on the device (d_ents[i].data_off/data_len
 * index it, data_len_total bytes); d_ents: n ewal_entry on the device.
 * d_out: device buffer of cap bytes.  *out_len = bytes written, *last_crc =
 * c_{n-1} (prev_crc when n == 0).  EWAL_E_NOMEM when the frames exceed cap,
 * EWAL_E_INVAL when an entry's payload lies outside d_data. */
int ewal_encode_entries_device(ewal_ctx *ctx, const void *d_data, uint64_t data_len_total, const ewal_entry *d_ents,
                               uint64_t n, uint32_t prev_crc, void *d_out, uint64_t cap, uint64_t *out_len,
                               uint32_t *last_crc);

/* Batched WAL writes on the GPU: a sequence of (*WAL).SaveState / SaveEntry /
 * Cut calls (wal/wal.go:219-279) encoded as ONE chained call.  Each record:
 *   EWAL_SAVE_ENTRY  SaveEntry(&Entry{Type: etype, Term: a, Index: b, Data})
 *   EWAL_SAVE_STATE  SaveState(&HardState{Term: a, Vote: b, Commit: c});
 *                    an empty HardState writes nothing (wal/wal.go:266-268)
 *   EWAL_SAVE_CUT    Cut's records: crcType{Crc: running CRC}, then
 *                    metadataType{Data: w.md} (wal/wal.go:232-237); Data is
 *                    the (data_off, data_len) bytes, or nil when data_nil
 * Data lives in d_data; d_recs on the device.  The frames go to d_out (cap
 * bytes): *out_len bytes, *last_crc the running CRC after the last record
 * (prev_crc when nothing was written).  h_rec_off (nullable, host, n
 * entries): the offset of each record's first frame in d_out -- a Cut's is
 * where the next file (walName(seq+1, enti+1)) starts.  Byte-identical to
 * the reference encoder (wal/encoder.go:25-37) over the same calls. */
#define EWAL_SAVE_ENTRY 2
#define EWAL_SAVE_STATE 3
#define EWAL_SAVE_CUT 4
typedef struct ewal_save_rec {
  int32_t kind;
  int32_t etype;
  uint64_t a, b, c;
  uint64_t data_off, data_len;
  int32_t data_nil;
  int32_t pad;
} ewal_save_rec;
int ewal_save_device(ewal_ctx *ctx, const void *d_data, uint64_t data_len_total, const ewal_save_rec *d_recs,
                     uint64_t n, uint32_t prev_crc, void *d_out, uint64_t cap, uint64_t *out_len, uint32_t *last_crc,
                     uint64_t *h_rec_off);

/* ---- CRC primitives (pkg/crc, pkg/crc/crc.go:23-41) ---------------------- */
/* crc32.Update(crc, MakeTable(poly), p) on a DEVICE buffer. */
int ewal_crc32_update_device(ewal_ctx *ctx, uint32_t crc, uint32_t poly, const void *d_buf, uint64_t n,
                             uint32_t *out);
/* crc32.Update on host memory (SSE4.2 for Castagnoli) -- for small writes. */
uint32_t ewal_crc32_update_host(uint32_t crc, uint32_t poly, const uint8_t *p, uint64_t n);
/* Update(c1, A || B) from c1=Update(0,A)... : returns Update(crc_a, B) given
 * crc_b = Update(0, B) and len_b, without touching the bytes. */
uint32_t ewal_crc32_combine(uint32_t poly, uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* ---- snapshots: snap.loadSnap / Snapshotter.Load, snap/snapshotter.go:62-111 */
/* Batch-verify snapshot FILES (snappb.Snapshot envelopes) resident in one
 * device buffer at offs[i], lens[i].  status[i] = EWAL_OK / EWAL_ERR_SNAP_CRC /
 * unmarshal class; crc outputs are the stored and recomputed CRCs. */
int esnap_verify_packed(ewal_ctx *ctx, const void *d_buf, uint64_t buf_len, const uint64_t *offs,
                        const uint64_t *lens, uint32_t n, uint32_t poly, int32_t *status,
                        uint32_t *stored_crc, uint32_t *computed_crc);
/* Snapshotter.Load(): newest-first over dir's *.snap, first success wins,
 * tried failures renamed *.broken.  On success *out_name (malloc'd, caller
 * frees with free()) names the snapshot file loaded; snapshot fields out.
 * Only the errors Go's loadSnap returns rename a file .broken; a Go panic
 * class (or EWAL_UNSUPPORTED_ENCODING: protobuf groups nested deeper than
 * the device walker's stack) stops Load with *out_name naming that file,
 * not renamed. */
typedef struct esnap_snapshot {
  uint64_t index, term;
  uint64_t data_off, data_len;   /* raftpb.Snapshot.Data within the file */
  int64_t n_nodes, n_removed;
  uint64_t nodes[64], removed[64];
} esnap_snapshot;
/* After esnap_verify_packed: the decoded raftpb.Snapshot of file i (only
 * meaningful when status[i] == EWAL_OK).  data_off == ~0: Data is not one
 * range of the file (several segments); n_nodes / n_removed > 64: only the
 * first 64 are held -- esnap_copy_field returns the full values. */
int esnap_copy_snapshot(ewal_ctx *ctx, uint32_t i, esnap_snapshot *out);
/* The full value of one raftpb.Snapshot field of file i of the last
 * esnap_verify_packed (d_buf still alive) or esnap_load_dir (i = 0): the
 * bytes of Data (the concatenation Go's append builds over repeated fields,
 * raft.pb.go:279-406) or of Snapshot.XXX_unrecognized, or the uint64 values
 * of Nodes / RemovedNodes.  Copies min(cap, full) bytes / values to out;
 * returns the full count or a negative error. */
enum { ESNAP_FIELD_DATA = 0, ESNAP_FIELD_UNREC = 1, ESNAP_FIELD_NODES = 2, ESNAP_FIELD_REMOVED = 3 };
int64_t esnap_copy_field(ewal_ctx *ctx, uint32_t i, int32_t field, void *out, int64_t cap);
int esnap_load_dir(ewal_ctx *ctx, const char *dirpath, uint32_t poly, esnap_snapshot *out, char **out_name);
/* Snapshotter.snapNames (snap/snapshotter.go:115-131): the *.snap names,
 * newest first, NUL-separated into out (cap bytes; *len = bytes needed).
 * Returns the count (0: ErrNoSnapshot) or a negative error. */
int64_t esnap_names(const char *dirpath, char *out, uint64_t cap, uint64_t *len);

/* ---- raft quorum commit: raft.maybeCommit, raft/raft.go:248-258 ---------- */
/* Batched over G independent raft groups (SoA).  match[v*G + g] for voter
 * v < nvoters[g] (1..255); log terms for group g are log_terms[log_ptr[g] ..
 * log_ptr[g+1]) at raft indices log_offset[g] + k.  committed[] is updated in
 * place; changed[g] = maybeCommit's return; status[g] = 0, or
 * EWAL_PANIC_BOUNDS where Go panics (no voters: mis[q-1] on an empty slice;
 * raftLog.at past the log).  All pointers are DEVICE pointers. */
int ecommit_batch_device(ewal_ctx *ctx, uint64_t G, const uint64_t *match, const uint8_t *nvoters,
                         const uint64_t *term, uint64_t *committed, const uint64_t *log_offset,
                         const uint64_t *log_ptr, const uint64_t *log_terms, uint8_t *changed,
                         uint8_t *status, double *device_ms);
/* The same maybeCommit over one 192-B record per group (the kernel reads
 * each group's state with coalesced loads instead of seven strided match
 * words plus a term gather that costs a whole line).  tail_term[k] is the
 * term of raftLog.ents[nlog-1-k] for k < min(13, nlog); when the quorum index lies
 * further back its term is read from log_terms[log_ptr[g] + (index -
 * log_offset)] (both may be NULL when the caller knows it never does: such a
 * group then gets status EWAL_UNSUPPORTED_ENCODING, as does a group with more
 * than 7 voters -- ecommit_batch_device takes those).  Outputs are SoA:
 * committed_out[g] (the new raftLog.committed), changed[g], status[g] as in
 * ecommit_batch_device.  All pointers are DEVICE pointers. */
typedef struct ecommit_group {
  uint64_t match[7];       /* Progress.Match of voters 0 .. nvoters-1 (raft/raft.go:252) */
  uint64_t committed;      /* raftLog.committed */
  uint64_t term;           /* raft.Term */
  uint64_t log_offset;     /* raftLog.offset: the index of ents[0] */
  uint32_t nlog;           /* len(raftLog.ents) */
  uint8_t nvoters;         /* 1..7 */
  uint8_t pad[3];
  uint64_t tail_term[13];  /* term of ents[nlog-1-k] */
} ecommit_group;
int ecommit_batch_rec_device(ewal_ctx *ctx, uint64_t G, const ecommit_group *groups, const uint64_t *log_ptr,
                             const uint64_t *log_terms, uint64_t *committed_out, uint8_t *changed,
                             uint8_t *status, double *device_ms);

/* ---- raft ingress: raftpb.Message.Unmarshal, raft/raftpb/raft.pb.go:407-617
 * (called per POST /raft in etcdserver/etcdhttp/http.go:119-146), batched
 * over n messages resident in one device buffer at offs[i], lens[i] (host
 * arrays).  status = EWAL_OK / EWAL_ERR_UNEXPECTED_EOF / EWAL_ERR_WRONG_TYPE /
 * EWAL_PANIC_BOUNDS / EWAL_NONTERMINATING as Unmarshal returns or panics
 * (EWAL_UNSUPPORTED_ENCODING only for protobuf groups nested deeper than the
 * device walker's stack).  The fields hold what Go leaves in the struct
 * (partial on error).  Entries go to a ctx-owned array: message i's are
 * [ents_first, ents_first + n_ents), fetched with emsg_copy_entries (Data
 * offsets are offsets into d_buf; data_nil == 2: Data is the concatenation
 * of that entry's EMSG_SEG_ENTRY_DATA segments).  The byte values Go builds
 * by append and the Snapshot's repeated fields are message i's segments
 * [segs_first, segs_first + n_segs) (emsg_copy_segments), in order:
 *   EMSG_SEG_UNREC         Message.XXX_unrecognized  (raft.pb.go:612-616)
 *   EMSG_SEG_ENTRY_UNREC   Entries[ent].XXX_unrecognized
 *   EMSG_SEG_ENTRY_DATA    Entries[ent].Data, repeated non-empty segments
 *   EMSG_SEG_SNAP_UNREC    Snapshot.XXX_unrecognized
 *   EMSG_SEG_SNAP_DATA     Snapshot.Data's segments (used when
 *                          snap_data_off == -2: a split field)
 *   EMSG_SEG_SNAP_NODE     one Snapshot.Nodes value (in off)
 *   EMSG_SEG_SNAP_REMOVED  one Snapshot.RemovedNodes value (in off)
 * a byte value is the concatenation of its kind's [off, off + len) ranges of
 * d_buf (none: nil). */
typedef struct emsg_message {
  int32_t status;
  int32_t reject;
  uint64_t type, to, from, term, log_term, index, commit;
  uint64_t ents_first, n_ents;
  uint64_t snap_index, snap_term;
  int64_t snap_data_off, snap_data_len;   /* Snapshot.Data in d_buf; off -1 == nil, -2: split (segments) */
  uint64_t snap_n_nodes, snap_n_removed;
  int64_t unrec_len;                       /* len(XXX_unrecognized) */
  uint64_t segs_first, n_segs;
} emsg_message;
enum {
  EMSG_SEG_UNREC = 0,
  EMSG_SEG_ENTRY_UNREC = 1,
  EMSG_SEG_ENTRY_DATA = 2,
  EMSG_SEG_SNAP_UNREC = 3,
  EMSG_SEG_SNAP_DATA = 4,
  EMSG_SEG_SNAP_NODE = 5,
  EMSG_SEG_SNAP_REMOVED = 6
};
typedef struct emsg_segment {
  int32_t kind;            /* EMSG_SEG_* */
  int32_t pad;
  int64_t ent;             /* the entry, counted within its message (EMSG_SEG_ENTRY_*), else -1 */
  uint64_t off, len;       /* a range of d_buf, or (value, 0) */
} emsg_segment;
int emsg_decode_batch_device(ewal_ctx *ctx, const void *d_buf, uint64_t buf_len, const uint64_t *offs,
                             const uint64_t *lens, uint32_t n, emsg_message *out, uint64_t *n_entries);
int64_t emsg_copy_entries(ewal_ctx *ctx, uint64_t first, ewal_entry *out, int64_t cap);
int64_t emsg_copy_segments(ewal_ctx *ctx, uint64_t first, emsg_segment *out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
