/* readall_shim.c -- the cgo shim of INTEGRATION.md ("readAllGPU"), in C.
 *
 * What a Go maintainer's `wal.OpenAtIndex(dir, index).ReadAll()` drop-in does
 * through the C ABI, step for step: create a context on a second thread (a
 * goroutine in Go) while the main one selects and opens the files
 * (ewal_open_at_index: wal/wal.go:108-159) and starts reading them
 * (ewal_wal_prefetch), then reserve the workspace for
 * their total size (ewal_ctx_reserve), ReadAll (ewal_wal_readall: the files
 * read and copied to HBM piece by piece, then the device pipeline,
 * wal/wal.go:164-216), then map the status to the
 * reference's sentinel / panic (the Go switch) and materialise the return
 * values the way the shim does: raftpb.Entry structs whose Data are
 * zero-copy views into the gathered WAL bytes, the metadata view, the
 * HardState, w.enti and the encoder seed (lastCRC), and every Entry's and
 * the HardState's XXX_unrecognized (raft.pb.go:273,699; fresh copies out of
 * the side list, as Go's Unmarshal appends them).
 *
 * Usage: readall_shim DIR INDEX [overlap|overlap-live]
 *   overlap       the ctx runs with EWAL_OPT_OVERLAP (two CU-masked streams)
 *   overlap-live  ... and the program exits WITHOUT ewal_ctx_destroy (the
 *                 library's atexit teardown of the masked streams, ewal.h)
 * prints one JSON line: the sentinel, the
 * result, a digest of ents (CRC-32C over each entry's (term, index, type,
 * nil, len, Data), the oracle's or_ents_digest format) and the time of each
 * step, and a digest of the XXX_unrecognized bytes (CRC-32C over (entry
 * index or ~0 for the HardState, len, bytes) of each non-nil one, in order).
 * Exit 0 whenever the call completed (whatever the sentinel).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <pthread.h>

#include "ewal.h"

/* raftpb.Entry as the shim materialises it (Go: {Type, Term, Index, Data []byte}) */
typedef struct {
  int32_t type;
  uint64_t term, index;
  const uint8_t *data;   /* NULL == nil; a view into the WAL bytes */
  uint64_t len;
  uint8_t *unrec;        /* XXX_unrecognized: NULL == nil; its own copy */
  uint64_t unrec_len;
} go_entry;

static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

/* the Go switch of readAllGPU: status -> the reference's value */
static const char *go_sentinel(int rc) {
  switch (rc) {
  case EWAL_OK: return "nil";
  case EWAL_ERR_UNEXPECTED_EOF: return "io.ErrUnexpectedEOF";
  case EWAL_ERR_RECORD_CRC: return "walpb.ErrCRCMismatch";
  case EWAL_ERR_WAL_CRC: return "wal.ErrCRCMismatch";
  case EWAL_ERR_METADATA_CONFLICT: return "wal.ErrMetadataConflict";
  case EWAL_ERR_INDEX_NOT_FOUND: return "wal.ErrIndexNotFound";
  case EWAL_ERR_WRONG_TYPE: return "proto.ErrWrongType";
  case EWAL_ERR_UNEXPECTED_TYPE: return "unexpected block type";
  case EWAL_ERR_FILE_NOT_FOUND: return "wal.ErrFileNotFound";
  case EWAL_UNSUPPORTED_ENCODING: return "fallback: Go decoder";
  default: return rc >= 32 ? "panic" : "infrastructure error";
  }
}

static uint32_t unrec_digest(uint32_t h, uint64_t who, const uint8_t *b, uint64_t n) {
  uint8_t hd[16];
  memcpy(hd, &who, 8);
  memcpy(hd + 8, &n, 8);
  h = ewal_crc32_update_host(h, 0x82F63B78u, hd, 16);
  return n ? ewal_crc32_update_host(h, 0x82F63B78u, b, n) : h;
}

static uint32_t ents_digest(const go_entry *e, int64_t n) {
  uint32_t h = 0;
  for (int64_t i = 0; i < n; i++) {
    uint8_t hd[32];
    const int32_t nil = e[i].data == NULL;
    memcpy(hd, &e[i].term, 8);
    memcpy(hd + 8, &e[i].index, 8);
    memcpy(hd + 16, &e[i].type, 4);
    memcpy(hd + 20, &nil, 4);
    memcpy(hd + 24, &e[i].len, 8);
    h = ewal_crc32_update_host(h, 0x82F63B78u, hd, 32);
    if (e[i].len) h = ewal_crc32_update_host(h, 0x82F63B78u, e[i].data, e[i].len);
  }
  return h;
}

/* the GPU context, created while the files are selected and read */
typedef struct {
  ewal_ctx *ctx;
  int rc;
  double t0, t1;
} ctx_job;
static void *make_ctx(void *arg) {
  ctx_job *j = (ctx_job *)arg;
  j->t0 = now_ms();
  j->rc = ewal_ctx_create(0, &j->ctx);
  j->t1 = now_ms();
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s DIR INDEX\n", argv[0]);
    return 2;
  }
  const uint64_t index = strtoull(argv[2], NULL, 0);
  const double t0 = now_ms();
  ctx_job job = {NULL, 0, 0, 0};
  pthread_t th;
  const int threaded = pthread_create(&th, NULL, make_ctx, &job) == 0;
  if (!threaded) make_ctx(&job);
  ewal_wal *w = NULL;
  int rc = ewal_open_at_index(argv[1], index, &w);        /* wal.OpenAtIndex: select + open the files */
  if (rc == 0) rc = ewal_wal_prefetch(w);                 /* ... and start reading them */
  const double t_open = now_ms();
  if (threaded) pthread_join(th, NULL);
  ewal_ctx *ctx = job.ctx;
  const double t2 = now_ms();                             /* context ready and the files opened */
  if (job.rc) {
    printf("{\"ok\": false, \"stage\": \"ctx\", \"rc\": %d, \"status\": \"%s\"}\n", job.rc,
           ewal_status_string(job.rc));
    return 0;
  }
  const int overlap = argc > 3 && strncmp(argv[3], "overlap", 7) == 0;
  const int keep_live = argc > 3 && strcmp(argv[3], "overlap-live") == 0;
  if (overlap && ewal_ctx_set_options(ctx, EWAL_OPT_OVERLAP) != EWAL_OK) {
    printf("{\"ok\": false, \"stage\": \"options\"}\n");
    return 0;
  }
  if (rc) {
    printf("{\"ok\": true, \"rc\": %d, \"sentinel\": \"%s\"}\n", rc, go_sentinel(rc));
    if (w) ewal_wal_close(w);
    ewal_ctx_destroy(ctx);
    return 0;
  }
  const uint64_t len = ewal_wal_size(w);
  rc = ewal_ctx_reserve(ctx, len, EWAL_RESERVE_HOST_STAGING);   /* sized from the directory listing */
  const double t3 = now_ms();
  if (rc) {
    printf("{\"ok\": false, \"stage\": \"reserve\", \"rc\": %d}\n", rc);
    return 0;
  }
  ewal_result r;
  rc = ewal_wal_readall(w, ctx, &r);                       /* (*WAL).ReadAll: read the files + HBM + verify */
  const double t4 = now_ms();
  const uint8_t *buf = ewal_wal_bytes(w, NULL);             /* the bytes ents are views into */
  /* materialise the Go return values */
  go_entry *ents = NULL;
  int64_t n = 0;
  uint8_t *state_unrec = NULL;   /* HardState.XXX_unrecognized */
  uint64_t state_unrec_len = 0;
  uint32_t udg = 0;
  uint64_t md_len = 0;
  const uint8_t *md = NULL;
  uint8_t *split = NULL;   /* split byte fields' concatenations (data_nil == 2, EWAL_FLAG_METADATA_SPLIT) */
  if (rc == EWAL_OK) {
    const int64_t ns = ewal_copy_split_bytes(ctx, NULL, 0);
    if (ns > 0) {
      split = (uint8_t *)malloc((size_t)ns);
      ewal_copy_split_bytes(ctx, split, ns);
    }
    if (r.metadata_off >= 0) {
      md = ((r.flags & EWAL_FLAG_METADATA_SPLIT) ? split : buf) + r.metadata_off;
      md_len = (uint64_t)r.metadata_len;
    }
    if (r.n_ents > 0) {
      ewal_entry *ds = (ewal_entry *)malloc(sizeof(ewal_entry) * (size_t)r.n_ents);
      n = ewal_copy_entries(ctx, ds, r.n_ents);
      ents = (go_entry *)malloc(sizeof(go_entry) * (size_t)(n > 0 ? n : 1));
      for (int64_t i = 0; i < n; i++) {
        ents[i].type = ds[i].type;
        ents[i].term = ds[i].term;
        ents[i].index = ds[i].index;
        ents[i].data = ds[i].data_nil == 0 ? buf + ds[i].data_off      /* zero-copy view */
                       : ds[i].data_nil == 2 ? split + ds[i].data_off   /* a split field's concatenation */
                       : NULL;
        ents[i].len = ds[i].data_len;
        ents[i].unrec = NULL;
        ents[i].unrec_len = 0;
      }
      free(ds);
    }
    if (r.n_unrec > 0) {   /* the side list: fresh XXX_unrecognized slices */
      ewal_unrec *u = (ewal_unrec *)malloc(sizeof(ewal_unrec) * r.n_unrec);
      const int64_t nu = ewal_copy_unrec(ctx, u, r.n_unrec);
      uint64_t tot = 0;
      for (int64_t i = 0; i < nu; i++)
        if (u[i].off + u[i].len > tot) tot = u[i].off + u[i].len;
      uint8_t *side = (uint8_t *)malloc(tot ? tot : 1);
      ewal_copy_unrec_bytes(ctx, side, (int64_t)tot);
      for (int64_t i = 0; i < nu; i++) {
        uint8_t *b = (uint8_t *)malloc(u[i].len ? u[i].len : 1);
        memcpy(b, side + u[i].off, u[i].len);
        if (u[i].ent < 0) {
          state_unrec = b;
          state_unrec_len = u[i].len;
        } else if (u[i].ent < n) {
          ents[u[i].ent].unrec = b;
          ents[u[i].ent].unrec_len = u[i].len;
        } else {
          free(b);
        }
      }
      free(side);
      free(u);
    }
    for (int64_t i = 0; i < n; i++)
      if (ents[i].unrec) udg = unrec_digest(udg, (uint64_t)i, ents[i].unrec, ents[i].unrec_len);
    if (state_unrec) udg = unrec_digest(udg, ~0ull, state_unrec, state_unrec_len);
  }
  const double t5 = now_ms();
  const uint32_t dg = ents_digest(ents, n);
  printf("{\"ok\": true, \"rc\": %d, \"sentinel\": \"%s\", \"status_string\": \"%s\", \"fail_record\": %lld, "
         "\"n_records\": %lld, \"n_ents\": %lld, \"flags\": %u, \"enti\": %llu, \"last_crc\": %u, \"has_state\": %d, "
         "\"state\": [%llu, %llu, %llu], \"metadata_len\": %lld, \"ents_digest\": %u, \"n_unrec\": %u, "
         "\"unrec_digest\": %u, \"wal_bytes\": %llu, "
         "\"ms\": {\"ctx_create\": %.3f, \"open_at_index\": %.3f, \"until_ctx_ready\": %.3f, \"reserve\": %.3f, "
         "\"readall\": %.3f, \"materialise\": %.3f, \"total\": %.3f}, \"device_ms\": %.3f, \"frames_ms\": %.3f}\n",
         rc, go_sentinel(rc), ewal_status_string(rc), (long long)r.fail_record, (long long)r.n_records,
         (long long)n, (unsigned)r.flags, (unsigned long long)r.enti, (unsigned)r.last_crc, r.has_state,
         (unsigned long long)r.state_term, (unsigned long long)r.state_vote, (unsigned long long)r.state_commit,
         md ? (long long)md_len : -1LL, dg, (unsigned)r.n_unrec, udg, (unsigned long long)len, job.t1 - job.t0,
         t_open - t0, t2 - t0, t3 - t2, t4 - t3, t5 - t4, t5 - t0, r.device_ms, r.frames_ms);
  for (int64_t i = 0; i < n; i++) free(ents[i].unrec);
  free(state_unrec);
  free(split);
  free(ents);
  ewal_wal_close(w);
  if (!keep_live) ewal_ctx_destroy(ctx);
  fflush(stdout);
  return 0;
}
