/*
 * ewal_cpu_fast.h -- the optimised CPU baseline (BASELINE.md "Optimised"
 * mode; see ewal_cpu_fast.c).  BASELINE/TEST INFRASTRUCTURE ONLY: bench.py's
 * cpu_baseline leg and tests/ load it, the product never does.
 */
#ifndef EWAL_CPU_FAST_H
#define EWAL_CPU_FAST_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORF_IRREGULAR 100   /* outside the fast path: use the faithful port */

typedef struct {             /* raftpb.Entry as a view into the WAL bytes */
  uint64_t term, index, data_off, data_len;
  int32_t type, data_nil;
} orf_ent;

typedef struct {
  int status;                /* OR_* (ewal_oracle.h) or ORF_IRREGULAR */
  int64_t detail, fail_record, fail_offset, n_records;
  uint32_t last_crc;
  uint64_t enti;
  int64_t metadata_off, metadata_len;   /* -1: nil */
  int has_state;
  uint64_t state_term, state_vote, state_commit;
  orf_ent *ents;
  int64_t n_ents;
} orf_result;

/* crc32.Update(crc, Castagnoli, p) with three interleaved SSE4.2 streams */
uint32_t orf_crc32c_update(uint32_t crc, const uint8_t *p, uint64_t n);
/* (*WAL).ReadAll (wal/wal.go:164-216) on nthreads cores */
int orf_readall(const uint8_t *buf, int64_t len, uint64_t ri, int nthreads, orf_result *out);
void orf_result_free(orf_result *r);
/* one WAL shard per worker: status and frames (n_records, or fail_record) */
void orf_readall_batch(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n, uint64_t ri,
                       int nthreads, int32_t *status, int64_t *frames);
/* the same with the faithful restatement (or_readall) per shard */
void orf_readall_batch_faithful(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n,
                                uint64_t ri, int nthreads, int32_t *status, int64_t *frames);
/* loadSnap's envelope + CRC check (snap/snapshotter.go:76-100), one file per worker */
void orf_snap_verify_batch(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n, int nthreads,
                           int32_t *status, uint32_t *computed);
/* raft.maybeCommit over group ranges (raft/raft.go:248-258), nthreads cores */
void orf_maybe_commit_batch(uint64_t G, const uint64_t *match, const uint8_t *nvoters, const uint64_t *term,
                            uint64_t *committed, const uint64_t *log_offset, const uint64_t *log_ptr,
                            const uint64_t *log_terms, uint8_t *changed, uint8_t *status, int nthreads);

/* OpenAtIndex(dir, ri).ReadAll() of a one-file WAL on the CPU, file read
 * included (nthreads readers; faithful: or_readall on 1 thread, else
 * orf_readall on nthreads): the status; frames, read and total ms out */
int orf_restart_file(const char *path, uint64_t ri, int nthreads, int faithful, int64_t *frames, double *read_ms,
                     double *total_ms);

/* raftpb.Message.Unmarshal (or_message_unmarshal) over n messages, strided over nthreads */
void orf_message_batch(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n, int nthreads,
                       int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
