/*
 * ewal_oracle.h -- CPU restatement of etcd's WAL replay-and-verify path.
 *
 * TEST INFRASTRUCTURE ONLY.  This oracle is the checker for the MI355X
 * engine in etcd_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product never links or calls it.
 *
 * Every function restates a Go function of the reference (mzsanford/etcd
 * v0.5.0-alpha, /root/reference) with Go's exact integer semantics (shifts
 * >= width yield 0, signed wrap-around, OR-accumulating repeated varint
 * fields, concatenating repeated bytes fields, empty bytes -> nil).
 * Citations are path:line relative to the reference root.
 *
 * Parity pinning: the reference is Go-only and no Go toolchain exists in
 * this image, so the oracle is pinned by the reference's own literal golden
 * bytes (wal/record_test.go:31-32), its known-answer tables
 * (raft/raft_test.go:465-504, wal/wal_test.go, snap/snapshotter_test.go) and
 * the RFC 3720 CRC-32C check value; see tests/test_oracle_golden.py.
 */
#ifndef EWAL_ORACLE_H
#define EWAL_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: identical numeric values to include/ewal.h (EWAL_*). */
enum {
  OR_OK = 0,
  OR_EOF = 1,                  /* io.EOF (clean end of stream; internal) */
  OR_ERR_UNEXPECTED_EOF = 2,   /* io.ErrUnexpectedEOF */
  OR_ERR_RECORD_CRC = 3,       /* walpb.ErrCRCMismatch  wal/walpb/record.go:22 */
  OR_ERR_WAL_CRC = 4,          /* wal.ErrCRCMismatch    wal/wal.go:48 */
  OR_ERR_METADATA_CONFLICT = 5,/* wal.ErrMetadataConflict wal/wal.go:45 */
  OR_ERR_INDEX_NOT_FOUND = 6,  /* wal.ErrIndexNotFound  wal/wal.go:47 */
  OR_ERR_WRONG_TYPE = 7,       /* proto.ErrWrongType    gogoprotobuf/proto/decode.go:49 */
  OR_ERR_UNEXPECTED_TYPE = 8,  /* fmt.Errorf("unexpected block type %d") wal/wal.go:194 */
  OR_ERR_FILE_NOT_FOUND = 9,   /* wal.ErrFileNotFound   wal/wal.go:46 */
  OR_ERR_SNAP_CRC = 10,        /* snap.ErrCRCMismatch   snap/snapshotter.go:25 */
  OR_ERR_NO_SNAPSHOT = 11,     /* snap.ErrNoSnapshot    snap/snapshotter.go:24 */
  OR_PANIC_NEG_LENGTH = 32,    /* make([]byte, l) with l < 0, wal/decoder.go:34 */
  OR_PANIC_BOUNDS = 33,        /* runtime slice/index bounds panic inside Unmarshal/Skip */
  OR_PANIC_ENTRY = 34,         /* mustUnmarshalEntry panic, wal/decoder.go:61-69 */
  OR_PANIC_STATE = 35,         /* mustUnmarshalState panic, wal/decoder.go:71-77 */
  OR_PANIC_INDEX_GAP = 36,     /* ents[:e.Index-ri] beyond len, wal/wal.go:173 */
  OR_NONTERMINATING = 37       /* reference never returns (loop / stack exhaustion) */
};

#define OR_CASTAGNOLI 0x82F63B78u
#define OR_IEEE 0xEDB88320u
#define OR_KOOPMAN 0xEB31D82Eu

/* ---- CRC-32 (Go hash/crc32) ------------------------------------------- */
/* crc32.Update(crc, MakeTable(poly), p): ^update(^crc, tab, p).
 * Call sites: pkg/crc/crc.go:32, snap/snapshotter.go:53,98. */
uint32_t or_crc32_update(uint32_t crc, uint32_t poly, const uint8_t *p, size_t n);
/* Same result via a portable byte-table loop (pins the SSE4.2 path). */
uint32_t or_crc32_update_table(uint32_t crc, uint32_t poly, const uint8_t *p, size_t n);

/* ---- protobuf messages ------------------------------------------------- */
typedef struct {
  int64_t type;
  uint32_t crc;
  uint8_t *data;      /* NULL == nil */
  int64_t data_len;
  int64_t unrec_len;  /* len(XXX_unrecognized) */
} or_record;

typedef struct {
  int32_t type;
  uint64_t term, index;
  uint8_t *data;      /* NULL == nil */
  int64_t data_len;
  int64_t unrec_len;
  uint8_t *unrec;     /* XXX_unrecognized (NULL == nil) */
} or_entry;

typedef struct {
  uint64_t term, vote, commit;
  int64_t unrec_len;
  uint8_t *unrec;     /* XXX_unrecognized (NULL == nil) */
} or_hardstate;

typedef struct {
  uint8_t *data; int64_t data_len;  /* NULL == nil */
  uint64_t *nodes; int64_t n_nodes;
  uint64_t index, term;
  uint64_t *removed; int64_t n_removed;
  int64_t unrec_len;
  uint8_t *unrec;     /* XXX_unrecognized (NULL == nil) */
} or_snapshot;

typedef struct {
  uint32_t crc;
  uint8_t *data; int64_t data_len;
  int64_t unrec_len;
} or_snappb;

/* raftpb.Message, raft/raftpb/raft.pb.go:125-137 */
typedef struct {
  uint64_t type, to, from, term, log_term, index, commit;
  int reject;
  or_entry *ents; int64_t n_ents;
  or_snapshot snap;
  int64_t unrec_len;
  uint8_t *unrec;     /* XXX_unrecognized (NULL == nil) */
} or_message;

/* Unmarshal: return OR_OK, OR_ERR_UNEXPECTED_EOF, OR_ERR_WRONG_TYPE,
 * OR_PANIC_BOUNDS or OR_NONTERMINATING.  The struct is left as Go leaves
 * it on error (partially filled); *_free releases owned buffers. */
int or_record_unmarshal(const uint8_t *d, int64_t l, or_record *m);     /* wal/walpb/record.pb.go:43-136 */
int or_entry_unmarshal(const uint8_t *d, int64_t l, or_entry *m);       /* raft/raftpb/raft.pb.go:170-277 */
int or_hardstate_unmarshal(const uint8_t *d, int64_t l, or_hardstate *m); /* raft/raftpb/raft.pb.go:618-704 */
int or_snapshot_unmarshal(const uint8_t *d, int64_t l, or_snapshot *m); /* raft/raftpb/raft.pb.go:279-406 */
int or_snappb_unmarshal(const uint8_t *d, int64_t l, or_snappb *m);     /* snap/snappb/snap.pb.go:42-120 */
/* proto.Skip, third_party/code.google.com/p/gogoprotobuf/proto/skip_gogo.go:33-116.
 * Returns status; *n receives the skip length on OR_OK. */
int or_proto_skip(const uint8_t *d, int64_t l, int64_t *n);
int or_message_unmarshal(const uint8_t *d, int64_t l, or_message *m);   /* raft/raftpb/raft.pb.go:407-617 */
void or_message_free(or_message *m);
/* Message.MarshalTo (raft.pb.go:1010-1068); ents = the n marshalled Entry
 * bodies back to back with their lengths, snap = marshalled Snapshot. */
int64_t or_message_marshal(uint64_t type, uint64_t to, uint64_t from, uint64_t term, uint64_t log_term,
                           uint64_t index, const uint8_t *ents, const int64_t *ent_lens, int64_t n_ents,
                           uint64_t commit, const uint8_t *snap, int64_t snap_len, int reject, uint8_t *out);
void or_record_free(or_record *m);
void or_entry_free(or_entry *m);
void or_hardstate_free(or_hardstate *m);
void or_snapshot_free(or_snapshot *m);
void or_snappb_free(or_snappb *m);

/* Marshal (MarshalTo) into out; returns bytes written.  out may be NULL to
 * query the size.  data==NULL encodes a nil field (omitted where Go omits). */
int64_t or_record_marshal(int64_t type, uint32_t crc, const uint8_t *data, int64_t n,
                          int data_nil, uint8_t *out);                   /* record.pb.go:175-196 */
int64_t or_entry_marshal(int32_t type, uint64_t term, uint64_t index,
                         const uint8_t *data, int64_t n, uint8_t *out);  /* raft.pb.go:921-943 */
int64_t or_hardstate_marshal(uint64_t term, uint64_t vote, uint64_t commit, uint8_t *out); /* raft.pb.go:1079-1097 */
int64_t or_snapshot_marshal(const uint8_t *data, int64_t n, const uint64_t *nodes, int64_t nn,
                            uint64_t index, uint64_t term, const uint64_t *removed, int64_t nr,
                            uint8_t *out);                               /* raft.pb.go:954-999 */
int64_t or_snappb_marshal(uint32_t crc, const uint8_t *data, int64_t n, int data_nil,
                          uint8_t *out);                                 /* snap.pb.go:158-176 */

/* ---- decoder / ReadAll ------------------------------------------------- */
typedef struct {
  const uint8_t *buf; int64_t len; int64_t pos;  /* bufio over MultiReader */
  uint32_t crc;                                  /* decoder.crc (pkg/crc digest) */
} or_decoder;

void or_decoder_init(or_decoder *d, const uint8_t *buf, int64_t len);  /* wal/decoder.go:20-26 */
/* decoder.decode, wal/decoder.go:28-47.  Returns OR_OK, OR_EOF, or an error/panic. */
int or_decode(or_decoder *d, or_record *rec);

typedef struct {
  int status;               /* OR_OK or the error/panic class */
  int64_t detail;           /* unexpected block type value, etc. */
  int64_t fail_record;      /* ordinal of the frame where it failed, -1 if none */
  int64_t fail_offset;      /* byte offset of that frame, -1 if none */
  int64_t n_records;        /* frames decoded before the end/failure */
  uint32_t last_crc;        /* decoder.lastCRC() (wal/decoder.go:53-55) on success */
  uint64_t enti;            /* w.enti */
  uint8_t *metadata; int64_t metadata_len;  /* NULL == nil */
  or_hardstate state; int has_state;
  or_entry *ents; int64_t n_ents;
} or_readall_result;

/* (*WAL).ReadAll over the concatenated bytes of names[nameIndex:] with
 * w.ri = ri, wal/wal.go:164-216. */
int or_readall(const uint8_t *buf, int64_t len, uint64_t ri, or_readall_result *out);
void or_readall_free(or_readall_result *r);

/* Per-record chained CRC listing: for each decoded frame, the decoder CRC
 * after it (decoder.crc.Sum32()).  Returns frames listed. */
int64_t or_chain_crcs(const uint8_t *buf, int64_t len, uint32_t *out, int64_t cap,
                      int64_t *offsets);

/* ---- encoder (write path, the generator) ------------------------------ */
typedef struct {
  uint8_t *buf; int64_t len, cap;
  uint32_t crc;             /* encoder.crc */
} or_encoder;
void or_encoder_init(or_encoder *e, uint32_t prev_crc);     /* wal/encoder.go:18-23 */
/* encoder.encode, wal/encoder.go:25-37 (rec.Crc is overwritten by the chain). */
int or_encode(or_encoder *e, int64_t type, const uint8_t *data, int64_t n, int data_nil);
void or_encoder_free(or_encoder *e);

/* ---- snapshot ---------------------------------------------------------- */
typedef struct {
  int status;               /* OR_OK, OR_ERR_SNAP_CRC, unmarshal errors/panics */
  uint32_t stored_crc, computed_crc;
  or_snapshot snap;
} or_loadsnap_result;
/* loadSnap content checks, snap/snapshotter.go:76-111, crcTable = poly. */
int or_loadsnap(const uint8_t *file, int64_t len, uint32_t poly, or_loadsnap_result *out);
void or_loadsnap_free(or_loadsnap_result *r);

/* ---- raft maybeCommit -------------------------------------------------- */
/* raft.maybeCommit (raft/raft.go:248-258, q() :275-277) followed by
 * raftLog.maybeCommit/term/at/isOutOfBounds (raft/log.go:115-154,194-217).
 * log_terms[k] = term of the entry at index offset+k (len(ents)=n_log).
 * Returns 1 if committed changed, 0 if not, -OR_PANIC_BOUNDS on the
 * reference's index-out-of-range panic (n_log==0 && offset==0). */
int or_maybe_commit(const uint64_t *match, int n, uint64_t term, uint64_t *committed,
                    const uint64_t *log_terms, uint64_t n_log, uint64_t offset);
void or_maybe_commit_batch(uint64_t G, const uint64_t *match, const uint8_t *nvoters, const uint64_t *term,
                           uint64_t *committed, const uint64_t *log_offset, const uint64_t *log_ptr,
                           const uint64_t *log_terms, uint8_t *changed, uint8_t *status);

/* ---- checker helpers (test infrastructure, not restatements) ----------- */
/* Digest of ReadAll's ents: CRC-32C over (type, term, index, nil, len, Data)
 * of every entry in order; the same digest over the engine's ewal_entry
 * descriptors (Data at buf + data_off). */
typedef struct { uint64_t term, index, data_off, data_len; int32_t type, data_nil; } or_ent_view;
uint32_t or_ents_digest(const or_readall_result *r);
uint32_t or_ent_views_digest(const uint8_t *buf, const or_ent_view *v, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
