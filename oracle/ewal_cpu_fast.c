/*
 * ewal_cpu_fast.c -- the OPTIMISED CPU baseline (BASELINE.md "Optimised"
 * mode): what a tuned CPU implementation of the same path reaches on the
 * GPU box's host cores.  BASELINE/TEST INFRASTRUCTURE ONLY: loaded by
 * bench.py's cpu_baseline leg and tests/, never by the product.
 *
 * Same results as the faithful restatement (ewal_oracle.c) on the inputs it
 * accepts; anything outside them returns ORF_IRREGULAR and the caller uses
 * or_readall / or_loadsnap instead (checked in tests/test_oracle_golden.py).
 *   - CRC-32C: three interleaved SSE4.2 crc32 streams per buffer, joined by
 *     the shift-by-n-zero-bytes tables (the register is GF(2)-linear), so
 *     the 3-cycle latency of the instruction is hidden (Go's own amd64
 *     castagnoliSSE42 does the same from Go 1.5 on; Go 1.3 ran one stream).
 *   - (*WAL).ReadAll (wal/wal.go:164-216): no per-record allocation (ents
 *     are views into the buffer), framing by one serial walk over the
 *     length prefixes (wal/decoder.go:79-83), then every frame's CRC in
 *     parallel on nthreads cores with the local-verify rule (frame i checks
 *     against frame i-1's stored Crc: equal to the running CRC up to the
 *     first failure, so the first failing frame is the reference's), then
 *     ReadAll's dispatch over the frame table.
 *   - batches: one shard / snapshot file per worker, all cores.
 */
#define _GNU_SOURCE
#include "ewal_cpu_fast.h"
#include "ewal_oracle.h"

#include <fcntl.h>
#include <nmmintrin.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ---- CRC-32C, 3 streams ------------------------------------------------ */
#define ORF_BLK 4096   /* bytes per stream per round */
static uint32_t g_shift_blk[4][256], g_shift_2blk[4][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

__attribute__((target("sse4.2"))) static uint32_t raw_crc(uint32_t c, const uint8_t *p, size_t n) {
  uint64_t r = c;
  while (n >= 8) { uint64_t v; memcpy(&v, p, 8); r = _mm_crc32_u64(r, v); p += 8; n -= 8; }
  while (n) { r = _mm_crc32_u8((uint32_t)r, *p++); n--; }
  return (uint32_t)r;
}

static void init_tables(void) {
  static uint8_t zeros[2 * ORF_BLK];
  for (int k = 0; k < 4; k++)
    for (int b = 0; b < 256; b++) {
      g_shift_blk[k][b] = raw_crc((uint32_t)b << (8 * k), zeros, ORF_BLK);
      g_shift_2blk[k][b] = raw_crc((uint32_t)b << (8 * k), zeros, 2 * ORF_BLK);
    }
}

static inline uint32_t shift_tab(const uint32_t (*t)[256], uint32_t x) {
  return t[0][x & 255] ^ t[1][(x >> 8) & 255] ^ t[2][(x >> 16) & 255] ^ t[3][x >> 24];
}

/* raw register update over p[0..n) (no pre/post inversion) */
__attribute__((target("sse4.2"))) static uint32_t raw_crc3(uint32_t c, const uint8_t *p, size_t n) {
  while (n >= 3 * ORF_BLK) {
    uint64_t a = c, b = 0, d = 0;
    const uint8_t *q = p;
    for (int i = 0; i < ORF_BLK; i += 8) {
      uint64_t x, y, z;
      memcpy(&x, q + i, 8);
      memcpy(&y, q + ORF_BLK + i, 8);
      memcpy(&z, q + 2 * ORF_BLK + i, 8);
      a = _mm_crc32_u64(a, x);
      b = _mm_crc32_u64(b, y);
      d = _mm_crc32_u64(d, z);
    }
    /* raw(c, A||B||C) = S_2L(raw(c, A)) ^ S_L(raw(0, B)) ^ raw(0, C) */
    c = shift_tab(g_shift_2blk, (uint32_t)a) ^ shift_tab(g_shift_blk, (uint32_t)b) ^ (uint32_t)d;
    p += 3 * ORF_BLK;
    n -= 3 * ORF_BLK;
  }
  return raw_crc(c, p, n);
}

uint32_t orf_crc32c_update(uint32_t crc, const uint8_t *p, uint64_t n) {
  pthread_once(&g_once, init_tables);
  return ~raw_crc3(~crc, p, (size_t)n);
}

/* ---- canonical varint / protobuf heads ---------------------------------- */
static inline int rd_varint(const uint8_t *p, int64_t end, int64_t *o, uint64_t *v) {
  uint64_t x = 0;
  for (int s = 0; s < 64; s += 7) {
    if (*o >= end) return 0;
    const uint8_t b = p[(*o)++];
    x |= (uint64_t)(b & 0x7f) << s;
    if (b < 0x80) { *v = x; return 1; }
  }
  return 0;
}

/* walpb.Record in MarshalTo's layout (record.pb.go:175-196):
 * 08 v(type) 10 v(crc) [1a v(n) data] -- exactly filling the frame. */
static int parse_record(const uint8_t *r, int64_t L, int64_t *type, uint32_t *crc, int64_t *doff, int64_t *dlen) {
  int64_t o = 0;
  uint64_t t, c, n;
  if (L < 4 || r[o++] != 0x08 || !rd_varint(r, L, &o, &t) || t >= 0x80) return 0;
  if (o >= L || r[o++] != 0x10 || !rd_varint(r, L, &o, &c) || c > 0xffffffffull) return 0;
  *type = (int64_t)t;
  *crc = (uint32_t)c;
  if (o == L) { *doff = 0; *dlen = 0; return 1; }
  if (r[o++] != 0x1a || !rd_varint(r, L, &o, &n) || n == 0 || n != (uint64_t)(L - o)) return 0;
  *doff = o;
  *dlen = (int64_t)n;
  return 1;
}

/* raftpb.Entry in MarshalTo's layout (raft.pb.go:921-943) */
static int parse_entry(const uint8_t *e, int64_t L, orf_ent *out) {
  int64_t o = 0;
  uint64_t t, term, idx, n;
  if (o >= L || e[o++] != 0x08 || !rd_varint(e, L, &o, &t) || t > 0x7fffffffull) return 0;
  if (o >= L || e[o++] != 0x10 || !rd_varint(e, L, &o, &term)) return 0;
  if (o >= L || e[o++] != 0x18 || !rd_varint(e, L, &o, &idx)) return 0;
  if (o >= L || e[o++] != 0x22 || !rd_varint(e, L, &o, &n) || n != (uint64_t)(L - o)) return 0;
  out->type = (int32_t)t;
  out->term = term;
  out->index = idx;
  out->data_off = (uint64_t)o;     /* relative; made absolute by the caller */
  out->data_len = n;
  out->data_nil = n == 0;
  return 1;
}

/* raftpb.HardState (raft.pb.go:1079-1097) */
static int parse_state(const uint8_t *s, int64_t L, uint64_t *term, uint64_t *vote, uint64_t *commit) {
  int64_t o = 0;
  if (o >= L || s[o++] != 0x08 || !rd_varint(s, L, &o, term)) return 0;
  if (o >= L || s[o++] != 0x10 || !rd_varint(s, L, &o, vote)) return 0;
  if (o >= L || s[o++] != 0x18 || !rd_varint(s, L, &o, commit)) return 0;
  return o == L;
}

/* ---- ReadAll ------------------------------------------------------------ */
typedef struct {
  uint64_t off, doff;
  int64_t dlen;
  int64_t type;
  uint32_t crc;
} frame_t;

typedef struct {
  const uint8_t *buf;
  const frame_t *fr;
  int64_t a, b;
  int64_t first_bad;   /* first frame in [a, b) whose check fails, or b */
} crc_job;

static void *crc_worker(void *arg) {
  crc_job *j = (crc_job *)arg;
  j->first_bad = j->b;
  for (int64_t i = j->a; i < j->b; i++) {
    const frame_t *f = &j->fr[i];
    if (f->type == 4) continue;   /* crcType: checked by ReadAll's seam rule */
    const uint32_t seed = i ? j->fr[i - 1].crc : 0u;
    const uint32_t c = f->dlen ? orf_crc32c_update(seed, j->buf + f->doff, (uint64_t)f->dlen) : seed;
    if (c != f->crc) { j->first_bad = i; break; }
  }
  return NULL;
}

int orf_readall(const uint8_t *buf, int64_t len, uint64_t ri, int nthreads, orf_result *out) {
  pthread_once(&g_once, init_tables);
  memset(out, 0, sizeof(*out));
  out->fail_record = -1;
  out->fail_offset = -1;
  out->metadata_off = -1;
  /* 1. framing: walk the length prefixes (wal/decoder.go:30-39) */
  int64_t cap = 1024, n = 0;
  frame_t *fr = (frame_t *)malloc(sizeof(frame_t) * (size_t)cap);
  int64_t p = 0;
  while (p < len) {
    if (len - p < 8) goto irregular;
    int64_t L;
    memcpy(&L, buf + p, 8);
    if (L < 0 || L > len - p - 8) goto irregular;
    if (n == cap) { cap *= 2; fr = (frame_t *)realloc(fr, sizeof(frame_t) * (size_t)cap); }
    frame_t *f = &fr[n];
    int64_t doff, dlen;
    if (!parse_record(buf + p + 8, L, &f->type, &f->crc, &doff, &dlen)) goto irregular;
    f->off = (uint64_t)p;
    f->doff = (uint64_t)(p + 8 + doff);
    f->dlen = dlen;
    n++;
    p += 8 + L;
  }
  /* 2. every frame's CRC check, nthreads ranges of about equal bytes */
  int64_t first_bad = n;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  {
    crc_job jobs[256];
    pthread_t th[256];
    int64_t at = 0;
    for (int t = 0; t < nthreads; t++) {
      const uint64_t want = (uint64_t)len * (uint64_t)(t + 1) / (uint64_t)nthreads;
      int64_t b = at;
      while (b < n && (t == nthreads - 1 || fr[b].off < want)) b++;
      jobs[t] = (crc_job){buf, fr, at, b, b};
      at = b;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, crc_worker, &jobs[t]);
    crc_worker(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < nthreads; t++)
      if (jobs[t].first_bad < jobs[t].b) { first_bad = jobs[t].first_bad; break; }
  }
  /* 3. ReadAll's dispatch (wal/wal.go:168-198) up to the first failure */
  int64_t ecap = 1024, ne = 0;
  orf_ent *ents = (orf_ent *)malloc(sizeof(orf_ent) * (size_t)ecap);
  uint64_t enti = 0;
  int64_t meta = -1;
  uint32_t running = 0;
  int st = OR_OK;
  int64_t i;
  for (i = 0; i < n; i++) {
    const frame_t *f = &fr[i];
    if (i == first_bad) { st = OR_ERR_RECORD_CRC; break; }
    if (f->type == 4) {
      if (running != 0 && f->crc != running) { st = OR_ERR_WAL_CRC; break; }
      running = f->crc;
      continue;
    }
    running = f->crc;
    if (f->type == 2) {
      orf_ent e;
      if (!parse_entry(buf + f->doff, f->dlen, &e)) goto irregular_e;
      e.data_off += f->doff;
      if (e.index >= ri) {
        const uint64_t k = e.index - ri;
        if (k > (uint64_t)ne) goto irregular_e;   /* index gap: the faithful port's panic class */
        ne = (int64_t)k;
        if (ne == ecap) { ecap *= 2; ents = (orf_ent *)realloc(ents, sizeof(orf_ent) * (size_t)ecap); }
        ents[ne++] = e;
        enti = e.index;
      } else {
        enti = e.index;
      }
    } else if (f->type == 3) {
      if (!parse_state(buf + f->doff, f->dlen, &out->state_term, &out->state_vote, &out->state_commit))
        goto irregular_e;
      out->has_state = 1;
    } else if (f->type == 1) {
      /* metadata != nil && !DeepEqual(metadata, rec.Data); metadata = rec.Data */
      if (meta >= 0 && fr[meta].dlen) {
        const frame_t *m = &fr[meta];
        if (f->dlen == 0 || m->dlen != f->dlen || memcmp(buf + m->doff, buf + f->doff, (size_t)f->dlen) != 0) {
          st = OR_ERR_METADATA_CONFLICT;
          break;
        }
      }
      meta = i;
    } else {
      st = OR_ERR_UNEXPECTED_TYPE;
      out->detail = f->type;
      break;
    }
  }
  out->n_records = i;
  out->enti = enti;
  if (st != OR_OK) {
    out->status = st;
    out->fail_record = i;
    out->fail_offset = (int64_t)fr[i].off;
    out->has_state = 0;
    free(ents);
    free(fr);
    return st;
  }
  if (enti < ri) {
    out->status = OR_ERR_INDEX_NOT_FOUND;
    out->has_state = 0;
    free(ents);
    free(fr);
    return out->status;
  }
  out->last_crc = running;
  if (meta >= 0 && fr[meta].dlen) {
    out->metadata_off = (int64_t)fr[meta].doff;
    out->metadata_len = fr[meta].dlen;
  }
  out->ents = ents;
  out->n_ents = ne;
  free(fr);
  return OR_OK;
irregular_e:
  free(ents);
irregular:
  free(fr);
  memset(out, 0, sizeof(*out));
  out->status = ORF_IRREGULAR;
  return ORF_IRREGULAR;
}

void orf_result_free(orf_result *r) {
  free(r->ents);
  r->ents = NULL;
  r->n_ents = 0;
}

/* ---- batches: one item per worker -------------------------------------- */
typedef struct {
  atomic_long next;
  int64_t n;
  int kind;   /* 0: WAL shards, 1: snapshot files, 2: WAL shards (faithful or_readall) */
  const uint8_t *buf;
  const uint64_t *offs, *lens;
  uint64_t ri;
  int32_t *status;
  int64_t *aux;
  uint32_t *aux32;
} batch_t;

/* snappb.Snapshot{Crc, Data} (snap.pb.go:158-176) + the CRC check of
 * loadSnap (snap/snapshotter.go:93-100); the raftpb.Snapshot body is not
 * decoded here (status OK = the CRC held) */
static int snap_crc(const uint8_t *f, int64_t L, uint32_t *computed) {
  int64_t o = 0;
  uint64_t c, n;
  if (o >= L || f[o++] != 0x08 || !rd_varint(f, L, &o, &c) || c > 0xffffffffull) return ORF_IRREGULAR;
  if (o >= L || f[o++] != 0x12 || !rd_varint(f, L, &o, &n) || n != (uint64_t)(L - o)) return ORF_IRREGULAR;
  *computed = orf_crc32c_update(0, f + o, n);
  return *computed == (uint32_t)c ? OR_OK : OR_ERR_SNAP_CRC;
}

static void *batch_worker(void *arg) {
  batch_t *b = (batch_t *)arg;
  for (;;) {
    const int64_t i = atomic_fetch_add(&b->next, 1);
    if (i >= b->n) break;
    const uint8_t *p = b->buf + b->offs[i];
    if (b->kind == 0) {
      orf_result r;
      b->status[i] = orf_readall(p, (int64_t)b->lens[i], b->ri, 1, &r);
      b->aux[i] = r.status == OR_OK ? r.n_records : r.fail_record;
      orf_result_free(&r);
    } else if (b->kind == 2) {   /* the faithful port, one shard per worker */
      or_readall_result r;
      b->status[i] = or_readall(p, (int64_t)b->lens[i], b->ri, &r);
      b->aux[i] = r.status == OR_OK ? r.n_records : r.fail_record;
      or_readall_free(&r);
    } else {
      b->status[i] = snap_crc(p, (int64_t)b->lens[i], &b->aux32[i]);
    }
  }
  return NULL;
}

static void run_batch(batch_t *b, int nthreads) {
  pthread_once(&g_once, init_tables);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  atomic_store(&b->next, 0);
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, b);
  batch_worker(b);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
}

void orf_readall_batch(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n, uint64_t ri,
                       int nthreads, int32_t *status, int64_t *frames) {
  batch_t b;
  memset(&b, 0, sizeof(b));
  b.n = n; b.kind = 0; b.buf = buf; b.offs = offs; b.lens = lens; b.ri = ri; b.status = status; b.aux = frames;
  run_batch(&b, nthreads);
}

void orf_readall_batch_faithful(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n,
                                uint64_t ri, int nthreads, int32_t *status, int64_t *frames) {
  batch_t b;
  memset(&b, 0, sizeof(b));
  b.n = n; b.kind = 2; b.buf = buf; b.offs = offs; b.lens = lens; b.ri = ri; b.status = status; b.aux = frames;
  run_batch(&b, nthreads);
}

void orf_snap_verify_batch(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n, int nthreads,
                           int32_t *status, uint32_t *computed) {
  batch_t b;
  memset(&b, 0, sizeof(b));
  b.n = n; b.kind = 1; b.buf = buf; b.offs = offs; b.lens = lens; b.status = status; b.aux32 = computed;
  run_batch(&b, nthreads);
}

/* ---- maybeCommit over group ranges ------------------------------------- */
typedef struct {
  uint64_t g0, g1, G;
  const uint64_t *match, *term, *log_offset, *log_ptr, *log_terms;
  const uint8_t *nvoters;
  uint64_t *committed;
  uint8_t *changed, *status;
} commit_job;

static void *commit_worker(void *arg) {
  commit_job *j = (commit_job *)arg;
  for (uint64_t g = j->g0; g < j->g1; g++) {
    uint64_t m[256];
    const int n = j->nvoters[g];
    for (int v = 0; v < n; v++) m[v] = j->match[(uint64_t)v * j->G + g];
    const int rc = or_maybe_commit(m, n, j->term[g], &j->committed[g], j->log_terms + j->log_ptr[g],
                                   j->log_ptr[g + 1] - j->log_ptr[g], j->log_offset[g]);
    j->status[g] = rc < 0 ? (uint8_t)(-rc) : 0;
    j->changed[g] = rc > 0 ? 1 : 0;
  }
  return NULL;
}

void orf_maybe_commit_batch(uint64_t G, const uint64_t *match, const uint8_t *nvoters, const uint64_t *term,
                            uint64_t *committed, const uint64_t *log_offset, const uint64_t *log_ptr,
                            const uint64_t *log_terms, uint8_t *changed, uint8_t *status, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  commit_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++)
    jobs[t] = (commit_job){G * (uint64_t)t / (uint64_t)nthreads, G * (uint64_t)(t + 1) / (uint64_t)nthreads, G,
                           match, term, log_offset, log_ptr, log_terms, nvoters, committed, changed, status};
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, commit_worker, &jobs[t]);
  commit_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
}


/* ---- the restart on the CPU, file reads included --------------------------
 * OpenAtIndex(dir, ri).ReadAll() of a one-file WAL as a CPU process does it:
 * read the file into memory (nthreads pread workers, 64 MiB pieces), then
 * ReadAll -- faithful: or_readall (the Go restatement, 1 thread); optimised:
 * orf_readall on nthreads cores.  The bench's restart cpu_baseline. */
typedef struct {
  int fd;
  uint8_t *buf;
  uint64_t size;
  atomic_uint_fast64_t *next;
  int err;
} read_job;
static void *read_worker(void *arg) {
  read_job *j = (read_job *)arg;
  const uint64_t piece = 64ull << 20;
  for (;;) {
    const uint64_t o = atomic_fetch_add(j->next, piece);
    if (o >= j->size) break;
    const uint64_t n = o + piece <= j->size ? piece : j->size - o;
    uint64_t got = 0;
    while (got < n) {
      const ssize_t r = pread(j->fd, j->buf + o + got, (size_t)(n - got), (off_t)(o + got));
      if (r <= 0) { j->err = 1; break; }
      got += (uint64_t)r;
    }
  }
  return NULL;
}
static double ms_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}
int orf_restart_file(const char *path, uint64_t ri, int nthreads, int faithful, int64_t *frames, double *read_ms,
                     double *total_ms) {
  const double t0 = ms_now();
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return -1; }
  const uint64_t size = (uint64_t)st.st_size;
  uint8_t *buf = (uint8_t *)malloc(size ? size : 1);
  if (!buf) { close(fd); return -1; }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  atomic_uint_fast64_t next;
  atomic_init(&next, 0);
  read_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) jobs[t] = (read_job){fd, buf, size, &next, 0};
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, read_worker, &jobs[t]);
  read_worker(&jobs[0]);
  int err = jobs[0].err;
  for (int t = 1; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    err |= jobs[t].err;
  }
  close(fd);
  const double t1 = ms_now();
  int status;
  if (err) {
    status = -1;
  } else if (faithful) {
    or_readall_result r;
    status = or_readall(buf, (int64_t)size, ri, &r);
    *frames = status == OR_OK ? r.n_records : r.fail_record;
    or_readall_free(&r);
  } else {
    orf_result r;
    status = orf_readall(buf, (int64_t)size, ri, nthreads, &r);
    *frames = status == OR_OK ? r.n_records : r.fail_record;
    orf_result_free(&r);
  }
  free(buf);
  *read_ms = t1 - t0;
  *total_ms = ms_now() - t0;
  return status;
}


/* ---- raftpb.Message.Unmarshal over a batch (the msg bench's cpu_baseline):
 * or_message_unmarshal + or_message_free per message, like Go's Unmarshal
 * into a fresh Message per POST /raft; messages strided over nthreads. */
typedef struct {
  const uint8_t *buf;
  const uint64_t *offs, *lens;
  int64_t n;
  int t, nt;
  int32_t *status;
} msg_job;
static void *msg_worker(void *arg) {
  msg_job *j = (msg_job *)arg;
  for (int64_t i = j->t; i < j->n; i += j->nt) {
    or_message m;
    j->status[i] = or_message_unmarshal(j->buf + j->offs[i], (int64_t)j->lens[i], &m);
    or_message_free(&m);
  }
  return NULL;
}
void orf_message_batch(const uint8_t *buf, const uint64_t *offs, const uint64_t *lens, int64_t n, int nthreads,
                       int32_t *status) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  msg_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) jobs[t] = (msg_job){buf, offs, lens, n, t, nthreads, status};
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, msg_worker, &jobs[t]);
  msg_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
}
