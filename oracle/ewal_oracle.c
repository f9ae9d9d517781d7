/*
 * ewal_oracle.c -- CPU restatement of etcd's WAL replay-and-verify path.
 * TEST INFRASTRUCTURE ONLY (see ewal_oracle.h).  Go semantics are restated
 * with explicit helpers: shl64/shl32 (Go shifts >= width give 0), wrapping
 * int64 adds via uint64, and byte-by-byte OR accumulation of varint fields.
 */
#include "ewal_oracle.h"
#include <stdlib.h>
#include <string.h>
#include <nmmintrin.h>

/* ===================================================================== */
/* CRC-32, Go hash/crc32                                                  */
/* ===================================================================== */
static uint32_t g_tab_poly[4];
static uint32_t g_tab[4][256];
static int g_ntab;

/* crc32.MakeTable: simpleMakeTable (reflected, LSB-first). */
static const uint32_t *get_table(uint32_t poly) {
  for (int i = 0; i < g_ntab; i++)
    if (g_tab_poly[i] == poly) return g_tab[i];
  int slot = g_ntab < 4 ? g_ntab++ : 3;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_tab[slot][i] = c;
  }
  g_tab_poly[slot] = poly;
  return g_tab[slot];
}

uint32_t or_crc32_update_table(uint32_t crc, uint32_t poly, const uint8_t *p, size_t n) {
  const uint32_t *t = get_table(poly);
  crc = ~crc;
  for (size_t i = 0; i < n; i++) crc = t[(uint8_t)crc ^ p[i]] ^ (crc >> 8);
  return ~crc;
}

/* Castagnoli via the SSE4.2 crc32 instruction, as Go's amd64 path does. */
__attribute__((target("sse4.2")))
static uint32_t crc32c_sse42(uint32_t crc, const uint8_t *p, size_t n) {
  uint64_t c = (uint32_t)~crc;
  while (n && ((uintptr_t)p & 7)) { c = _mm_crc32_u8((uint32_t)c, *p++); n--; }
  while (n >= 8) { uint64_t v; memcpy(&v, p, 8); c = _mm_crc32_u64(c, v); p += 8; n -= 8; }
  while (n) { c = _mm_crc32_u8((uint32_t)c, *p++); n--; }
  return ~(uint32_t)c;
}

uint32_t or_crc32_update(uint32_t crc, uint32_t poly, const uint8_t *p, size_t n) {
  if (poly == OR_CASTAGNOLI && __builtin_cpu_supports("sse4.2")) return crc32c_sse42(crc, p, n);
  return or_crc32_update_table(crc, poly, p, n);
}

/* ===================================================================== */
/* Go integer helpers                                                     */
/* ===================================================================== */
static inline uint64_t shl64(uint64_t x, uint64_t s) { return s >= 64 ? 0 : x << s; }
static inline uint32_t shl32(uint32_t x, uint64_t s) { return s >= 32 ? 0 : x << s; }
static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t le64(const uint8_t *p) { int64_t v; memcpy(&v, p, 8); return v; }

/* append(dst, src...) on a Go []byte held as (ptr,len); nil stays nil when
 * nothing is appended. */
static void bytes_append(uint8_t **dst, int64_t *dlen, const uint8_t *src, int64_t n) {
  if (n <= 0) return;
  *dst = (uint8_t *)realloc(*dst, (size_t)(*dlen + n));
  memcpy(*dst + *dlen, src, (size_t)n);
  *dlen += n;
}
static void u64_append(uint64_t **dst, int64_t *n, uint64_t v) {
  *dst = (uint64_t *)realloc(*dst, (size_t)(*n + 1) * sizeof(uint64_t));
  (*dst)[(*n)++] = v;
}

/* ===================================================================== */
/* proto.Skip  (skip_gogo.go:33-116), iterative restatement               */
/* ===================================================================== */
/* The recursion of case 3 (start group) is kept as an explicit stack of
 * frames.  Frame = Skip(data[base:]) with its local index.  Two exact
 * non-termination tests: a frame whose loop runs more iterations than it
 * has positions must revisit a position (deterministic => cycles forever),
 * and a child pushed at local start 0 re-enters its own parent (infinite
 * recursion).  Depth beyond Go's 1 GB goroutine stack is reported as
 * non-terminating too (boundary approximate: ~200 B per Skip frame). */
#define SKIP_MAX_DEPTH 5000000
typedef struct { int64_t base, idx, start, iters; } skframe;

static int skip_read_wire(const uint8_t *d, int64_t l, int64_t *idx, uint64_t *wire) {
  uint64_t w = 0;
  for (uint64_t shift = 0;; shift += 7) {
    if (*idx >= l) return OR_ERR_UNEXPECTED_EOF;
    if (*idx < 0) return OR_PANIC_BOUNDS;   /* data[index] with index < 0 */
    uint8_t b = d[(*idx)++];
    w |= shl64((uint64_t)(b & 0x7F), shift);
    if (b < 0x80) break;
  }
  *wire = w;
  return OR_OK;
}

/* Skip for a single non-group field whose tag has already been read:
 * idx is local (after the tag).  Returns the Skip return value. */
static int skip_simple(const uint8_t *d, int64_t l, int wt, int64_t idx, int64_t *n) {
  switch (wt) {
  case 0:
    for (;;) {
      if (idx >= l) return OR_ERR_UNEXPECTED_EOF;
      idx++;
      if (d[idx - 1] < 0x80) break;
    }
    *n = idx; return OR_OK;
  case 1: *n = wadd(idx, 8); return OR_OK;
  case 2: {
    int64_t length = 0;
    for (uint64_t shift = 0;; shift += 7) {
      if (idx >= l) return OR_ERR_UNEXPECTED_EOF;
      uint8_t b = d[idx++];
      length = (int64_t)((uint64_t)length | shl64((uint64_t)(b & 0x7F), shift));
      if (b < 0x80) break;
    }
    *n = wadd(idx, length); return OR_OK;
  }
  case 4: *n = idx; return OR_OK;
  case 5: *n = wadd(idx, 4); return OR_OK;
  default: return OR_ERR_WRONG_TYPE;
  }
}

int or_proto_skip(const uint8_t *d0, int64_t l0, int64_t *out) {
  if (l0 <= 0) return OR_PANIC_BOUNDS; /* panic("unreachable") */
  int64_t idx = 0;
  uint64_t wire;
  int st = skip_read_wire(d0, l0, &idx, &wire);
  if (st) return st;
  int wt = (int)(wire & 7);
  if (wt != 3) return skip_simple(d0, l0, wt, idx, out);

  /* group: frame stack */
  int64_t cap = 16, depth = 0;
  skframe *stk = (skframe *)malloc(sizeof(skframe) * cap);
  skframe cur = {0, idx, 0, 0};
  for (;;) {
    const uint8_t *d = d0 + cur.base;
    int64_t l = l0 - cur.base;
    if (++cur.iters > l + 1) { st = OR_NONTERMINATING; break; }
    int64_t start = cur.idx;
    int64_t j = cur.idx;
    st = skip_read_wire(d, l, &j, &wire);
    if (st) break;
    int wt2 = (int)(wire & 7);
    if (wt2 == 4) {
      /* break out of this frame's loop: return index j */
      int64_t ret = j;
      if (depth == 0) { *out = ret; st = OR_OK; break; }
      cur = stk[--depth];
      cur.idx = wadd(cur.start, ret);
      continue;
    }
    if (wt2 == 3) {
      /* next, err := Skip(data[start:]) -- recursion into a new group */
      if (start == 0) { st = OR_NONTERMINATING; break; }
      if (depth + 1 >= SKIP_MAX_DEPTH) { st = OR_NONTERMINATING; break; }
      if (depth == cap) { cap *= 2; stk = (skframe *)realloc(stk, sizeof(skframe) * cap); }
      cur.start = start;
      stk[depth++] = cur;
      skframe child = {cur.base + start, j - start, 0, 0};
      cur = child;
      continue;
    }
    /* simple child: Skip(data[start:]) re-reads the same tag */
    int64_t n;
    st = skip_simple(d + start, l - start, wt2, j - start, &n);
    if (st) break;
    cur.idx = wadd(start, n);
  }
  free(stk);
  return st;
}

/* ===================================================================== */
/* Generic gogoprotobuf Unmarshal engine                                  */
/* ===================================================================== */
enum { F_U64, F_I64, F_U32, F_I32, F_BYTES, F_U64REP };
typedef struct {
  int num, kind;
  void *p;            /* target scalar, or uint8_t** / uint64_t** */
  int64_t *plen;      /* bytes length / repeated count */
} fspec;

/* unknown fields: Skip, then `m.XXX_unrecognized = append(m.XXX_unrecognized,
 * data[index:index+skippy]...)` (e.g. raft.pb.go:270); unrec may be NULL for
 * messages whose XXX_unrecognized the path never returns. */
static int pb_unmarshal(const uint8_t *d, int64_t l, fspec *fs, int nf, int64_t *unrec_len, uint8_t **unrec) {
  int64_t index = 0;
  while (index < l) {
    uint64_t wire = 0;
    for (uint64_t shift = 0;; shift += 7) {
      if (index >= l) return OR_ERR_UNEXPECTED_EOF;
      uint8_t b = d[index++];
      wire |= shl64((uint64_t)(b & 0x7F), shift);
      if (b < 0x80) break;
    }
    int32_t fieldNum = (int32_t)(uint32_t)(wire >> 3);
    int wireType = (int)(wire & 7);
    fspec *f = NULL;
    for (int i = 0; i < nf; i++) if (fs[i].num == fieldNum) { f = &fs[i]; break; }
    if (f) {
      if (f->kind == F_BYTES) {
        if (wireType != 2) return OR_ERR_WRONG_TYPE;
        int64_t byteLen = 0;
        for (uint64_t shift = 0;; shift += 7) {
          if (index >= l) return OR_ERR_UNEXPECTED_EOF;
          uint8_t b = d[index++];
          byteLen = (int64_t)((uint64_t)byteLen | shl64((uint64_t)(b & 0x7F), shift));
          if (b < 0x80) break;
        }
        int64_t postIndex = wadd(index, byteLen);
        if (postIndex > l) return OR_ERR_UNEXPECTED_EOF;
        if (postIndex < index) return OR_PANIC_BOUNDS;  /* data[index:postIndex] */
        bytes_append((uint8_t **)f->p, f->plen, d + index, postIndex - index);
        index = postIndex;
        continue;
      }
      if (wireType != 0) return OR_ERR_WRONG_TYPE;
      uint64_t v = 0;
      for (uint64_t shift = 0;; shift += 7) {
        if (index >= l) return OR_ERR_UNEXPECTED_EOF;
        uint8_t b = d[index++];
        switch (f->kind) {
        case F_U64: *(uint64_t *)f->p |= shl64((uint64_t)(b & 0x7F), shift); break;
        case F_I64: *(int64_t *)f->p = (int64_t)((uint64_t)*(int64_t *)f->p | shl64((uint64_t)(b & 0x7F), shift)); break;
        case F_U32: *(uint32_t *)f->p |= shl32((uint32_t)(b & 0x7F), shift); break;
        case F_I32: *(int32_t *)f->p = (int32_t)((uint32_t)*(int32_t *)f->p | shl32((uint32_t)(b & 0x7F), shift)); break;
        case F_U64REP: v |= shl64((uint64_t)(b & 0x7F), shift); break;
        }
        if (b < 0x80) break;
      }
      if (f->kind == F_U64REP) u64_append((uint64_t **)f->p, f->plen, v);
      continue;
    }
    /* default: unknown field -> Skip into XXX_unrecognized */
    int64_t sizeOfWire = 0;
    uint64_t w = wire;
    do { sizeOfWire++; w >>= 7; } while (w != 0);
    index -= sizeOfWire;
    int64_t skippy;
    int st = or_proto_skip(d + index, l - index, &skippy);
    if (st) return st;
    int64_t hi = wadd(index, skippy);
    if (hi > l) return OR_ERR_UNEXPECTED_EOF;
    if (hi < index) return OR_PANIC_BOUNDS;      /* data[index:index+skippy] */
    if (skippy == 0) return OR_NONTERMINATING;   /* index never advances */
    if (unrec) bytes_append(unrec, unrec_len, d + index, skippy);
    else *unrec_len += skippy;
    index = hi;
  }
  return OR_OK;
}

int or_record_unmarshal(const uint8_t *d, int64_t l, or_record *m) {
  fspec fs[3] = {{1, F_I64, &m->type, 0}, {2, F_U32, &m->crc, 0}, {3, F_BYTES, &m->data, &m->data_len}};
  return pb_unmarshal(d, l, fs, 3, &m->unrec_len, NULL);
}
int or_entry_unmarshal(const uint8_t *d, int64_t l, or_entry *m) {
  fspec fs[4] = {{1, F_I32, &m->type, 0}, {2, F_U64, &m->term, 0}, {3, F_U64, &m->index, 0},
                 {4, F_BYTES, &m->data, &m->data_len}};
  return pb_unmarshal(d, l, fs, 4, &m->unrec_len, &m->unrec);
}
int or_hardstate_unmarshal(const uint8_t *d, int64_t l, or_hardstate *m) {
  fspec fs[3] = {{1, F_U64, &m->term, 0}, {2, F_U64, &m->vote, 0}, {3, F_U64, &m->commit, 0}};
  return pb_unmarshal(d, l, fs, 3, &m->unrec_len, &m->unrec);
}
int or_snapshot_unmarshal(const uint8_t *d, int64_t l, or_snapshot *m) {
  fspec fs[5] = {{1, F_BYTES, &m->data, &m->data_len}, {2, F_U64REP, &m->nodes, &m->n_nodes},
                 {3, F_U64, &m->index, 0}, {4, F_U64, &m->term, 0},
                 {5, F_U64REP, &m->removed, &m->n_removed}};
  return pb_unmarshal(d, l, fs, 5, &m->unrec_len, &m->unrec);
}
int or_snappb_unmarshal(const uint8_t *d, int64_t l, or_snappb *m) {
  fspec fs[2] = {{1, F_U32, &m->crc, 0}, {2, F_BYTES, &m->data, &m->data_len}};
  return pb_unmarshal(d, l, fs, 2, &m->unrec_len, NULL);
}

/* raftpb.Message.Unmarshal, raft/raftpb/raft.pb.go:407-617.  Quirks kept:
 * an Entry's Unmarshal error is discarded (:535, the return value is not
 * checked) but a panic inside it propagates; Snapshot errors return (:575);
 * Reject is assigned (v != 0), not OR-ed (:593); repeated Snapshot fields
 * accumulate into the same struct. */
static int msg_varint(const uint8_t *d, int64_t *index, int64_t l, uint64_t *v) {
  for (uint64_t shift = 0;; shift += 7) {
    if (*index >= l) return OR_ERR_UNEXPECTED_EOF;
    uint8_t b = d[(*index)++];
    *v |= shl64((uint64_t)(b & 0x7F), shift);
    if (b < 0x80) return OR_OK;
  }
}
int or_message_unmarshal(const uint8_t *d, int64_t l, or_message *m) {
  int64_t index = 0;
  while (index < l) {
    uint64_t wire = 0;
    if (msg_varint(d, &index, l, &wire)) return OR_ERR_UNEXPECTED_EOF;
    int32_t fieldNum = (int32_t)(uint32_t)(wire >> 3);
    int wireType = (int)(wire & 7);
    uint64_t *u = NULL;
    switch (fieldNum) {
    case 1: u = &m->type; break;
    case 2: u = &m->to; break;
    case 3: u = &m->from; break;
    case 4: u = &m->term; break;
    case 5: u = &m->log_term; break;
    case 6: u = &m->index; break;
    case 8: u = &m->commit; break;
    default: break;
    }
    if (u) {
      if (wireType != 0) return OR_ERR_WRONG_TYPE;
      if (msg_varint(d, &index, l, u)) return OR_ERR_UNEXPECTED_EOF;
      continue;
    }
    if (fieldNum == 7 || fieldNum == 9) {
      if (wireType != 2) return OR_ERR_WRONG_TYPE;
      uint64_t ml = 0;
      if (msg_varint(d, &index, l, &ml)) return OR_ERR_UNEXPECTED_EOF;
      int64_t postIndex = wadd(index, (int64_t)ml);
      if (postIndex > l) return OR_ERR_UNEXPECTED_EOF;
      if (postIndex < index) return OR_PANIC_BOUNDS;   /* data[index:postIndex] */
      if (fieldNum == 7) {
        m->ents = (or_entry *)realloc(m->ents, sizeof(or_entry) * (size_t)(m->n_ents + 1));
        or_entry *e = &m->ents[m->n_ents++];
        memset(e, 0, sizeof(*e));
        int st = or_entry_unmarshal(d + index, postIndex - index, e);
        if (st == OR_PANIC_BOUNDS || st == OR_NONTERMINATING) return st;   /* panics propagate */
      } else {
        int st = or_snapshot_unmarshal(d + index, postIndex - index, &m->snap);
        if (st) return st;
      }
      index = postIndex;
      continue;
    }
    if (fieldNum == 10) {
      if (wireType != 0) return OR_ERR_WRONG_TYPE;
      uint64_t v = 0;
      if (msg_varint(d, &index, l, &v)) return OR_ERR_UNEXPECTED_EOF;
      m->reject = v != 0;
      continue;
    }
    int64_t sizeOfWire = 0;
    uint64_t w = wire;
    do { sizeOfWire++; w >>= 7; } while (w != 0);
    index -= sizeOfWire;
    int64_t skippy;
    int st = or_proto_skip(d + index, l - index, &skippy);
    if (st) return st;
    int64_t hi = wadd(index, skippy);
    if (hi > l) return OR_ERR_UNEXPECTED_EOF;
    if (hi < index) return OR_PANIC_BOUNDS;
    if (skippy == 0) return OR_NONTERMINATING;
    bytes_append(&m->unrec, &m->unrec_len, d + index, skippy);   /* m.XXX_unrecognized = append(...) */
    index = hi;
  }
  return OR_OK;
}
void or_message_free(or_message *m) {
  free(m->unrec);
  for (int64_t i = 0; i < m->n_ents; i++) or_entry_free(&m->ents[i]);
  free(m->ents);
  or_snapshot_free(&m->snap);
  memset(m, 0, sizeof(*m));
}

void or_record_free(or_record *m) { free(m->data); memset(m, 0, sizeof(*m)); }
void or_entry_free(or_entry *m) { free(m->data); free(m->unrec); memset(m, 0, sizeof(*m)); }
void or_hardstate_free(or_hardstate *m) { free(m->unrec); memset(m, 0, sizeof(*m)); }
void or_snapshot_free(or_snapshot *m) {
  free(m->data); free(m->nodes); free(m->removed); free(m->unrec);
  memset(m, 0, sizeof(*m));
}
void or_snappb_free(or_snappb *m) { free(m->data); memset(m, 0, sizeof(*m)); }

/* ===================================================================== */
/* Marshal                                                                */
/* ===================================================================== */
static int64_t put_varint(uint8_t *out, int64_t i, uint64_t v) {
  while (v >= 0x80) { if (out) out[i] = (uint8_t)(v | 0x80); v >>= 7; i++; }
  if (out) out[i] = (uint8_t)v;
  return i + 1;
}
static int64_t put_byte(uint8_t *out, int64_t i, uint8_t b) { if (out) out[i] = b; return i + 1; }
static int64_t put_bytes(uint8_t *out, int64_t i, const uint8_t *p, int64_t n) {
  if (out && n) memcpy(out + i, p, (size_t)n);
  return i + n;
}

int64_t or_record_marshal(int64_t type, uint32_t crc, const uint8_t *data, int64_t n, int data_nil, uint8_t *out) {
  int64_t i = 0;
  i = put_byte(out, i, 0x08); i = put_varint(out, i, (uint64_t)type);
  i = put_byte(out, i, 0x10); i = put_varint(out, i, (uint64_t)crc);
  if (!data_nil) { i = put_byte(out, i, 0x1a); i = put_varint(out, i, (uint64_t)n); i = put_bytes(out, i, data, n); }
  return i;
}
int64_t or_entry_marshal(int32_t type, uint64_t term, uint64_t index, const uint8_t *data, int64_t n, uint8_t *out) {
  int64_t i = 0;
  i = put_byte(out, i, 0x08); i = put_varint(out, i, (uint64_t)(int64_t)type);
  i = put_byte(out, i, 0x10); i = put_varint(out, i, term);
  i = put_byte(out, i, 0x18); i = put_varint(out, i, index);
  i = put_byte(out, i, 0x22); i = put_varint(out, i, (uint64_t)n); i = put_bytes(out, i, data, n);
  return i;
}
int64_t or_hardstate_marshal(uint64_t term, uint64_t vote, uint64_t commit, uint8_t *out) {
  int64_t i = 0;
  i = put_byte(out, i, 0x08); i = put_varint(out, i, term);
  i = put_byte(out, i, 0x10); i = put_varint(out, i, vote);
  i = put_byte(out, i, 0x18); i = put_varint(out, i, commit);
  return i;
}
int64_t or_snapshot_marshal(const uint8_t *data, int64_t n, const uint64_t *nodes, int64_t nn, uint64_t index,
                            uint64_t term, const uint64_t *removed, int64_t nr, uint8_t *out) {
  int64_t i = 0;
  i = put_byte(out, i, 0x0a); i = put_varint(out, i, (uint64_t)n); i = put_bytes(out, i, data, n);
  for (int64_t k = 0; k < nn; k++) { i = put_byte(out, i, 0x10); i = put_varint(out, i, nodes[k]); }
  i = put_byte(out, i, 0x18); i = put_varint(out, i, index);
  i = put_byte(out, i, 0x20); i = put_varint(out, i, term);
  for (int64_t k = 0; k < nr; k++) { i = put_byte(out, i, 0x28); i = put_varint(out, i, removed[k]); }
  return i;
}
int64_t or_snappb_marshal(uint32_t crc, const uint8_t *data, int64_t n, int data_nil, uint8_t *out) {
  int64_t i = 0;
  i = put_byte(out, i, 0x08); i = put_varint(out, i, (uint64_t)crc);
  if (!data_nil) { i = put_byte(out, i, 0x12); i = put_varint(out, i, (uint64_t)n); i = put_bytes(out, i, data, n); }
  return i;
}

/* ===================================================================== */
/* decoder.decode (wal/decoder.go:28-47)                                  */
/* ===================================================================== */
void or_decoder_init(or_decoder *d, const uint8_t *buf, int64_t len) {
  d->buf = buf; d->len = len; d->pos = 0; d->crc = 0;   /* crc.New(0, crcTable) */
}

int or_decode(or_decoder *d, or_record *rec) {
  or_record_free(rec);                                   /* rec.Reset() */
  int64_t rem = d->len - d->pos;
  /* readInt64: binary.Read -> io.ReadFull of 8 bytes */
  if (rem == 0) return OR_EOF;
  if (rem < 8) { d->pos = d->len; return OR_ERR_UNEXPECTED_EOF; }
  int64_t l = le64(d->buf + d->pos);
  d->pos += 8; rem -= 8;
  if (l < 0) return OR_PANIC_NEG_LENGTH;                 /* make([]byte, l) */
  /* io.ReadFull(d.br, data): 0 bytes read -> io.EOF, some -> ErrUnexpectedEOF.
   * (A length beyond host memory makes Go's make() fail first; not modelled.) */
  if (l > rem) { d->pos = d->len; return rem == 0 ? OR_EOF : OR_ERR_UNEXPECTED_EOF; }
  const uint8_t *data = d->buf + d->pos;
  d->pos += l;
  int st = or_record_unmarshal(data, l, rec);
  if (st) return st;
  if (rec->type == 4) return OR_OK;                      /* crcType: skip the check */
  d->crc = or_crc32_update(d->crc, OR_CASTAGNOLI, rec->data, (size_t)rec->data_len);
  if (rec->crc == d->crc) return OR_OK;                  /* rec.Validate */
  or_record_free(rec);
  return OR_ERR_RECORD_CRC;
}

/* ===================================================================== */
/* (*WAL).ReadAll (wal/wal.go:164-216)                                    */
/* ===================================================================== */
static int panic_class(int st, int cls) {
  /* mustUnmarshal* panics with the Unmarshal error; runtime panics and
   * non-termination keep their own class. */
  if (st == OR_PANIC_BOUNDS || st == OR_NONTERMINATING) return st;
  return cls;
}

int or_readall(const uint8_t *buf, int64_t len, uint64_t ri, or_readall_result *out) {
  memset(out, 0, sizeof(*out));
  out->fail_record = -1; out->fail_offset = -1;
  or_decoder dec; or_decoder_init(&dec, buf, len);
  or_record rec; memset(&rec, 0, sizeof(rec));
  uint8_t *metadata = NULL; int64_t mlen = 0;
  or_hardstate state; memset(&state, 0, sizeof(state)); int has_state = 0;
  or_entry *ents = NULL; int64_t n_ents = 0, cap_ents = 0;
  uint64_t enti = 0;
  int64_t nrec = 0;
  int st;
  int64_t frame_off = 0;
  for (;;) {
    frame_off = dec.pos;
    st = or_decode(&dec, &rec);
    if (st != OR_OK) break;
    switch (rec.type) {
    case 2: { /* entryType */
      or_entry e; memset(&e, 0, sizeof(e));
      int s2 = or_entry_unmarshal(rec.data, rec.data_len, &e);
      if (s2) { or_entry_free(&e); st = panic_class(s2, OR_PANIC_ENTRY); goto fail; }
      if (e.index >= ri) {
        uint64_t k = e.index - ri;
        if (k > (uint64_t)n_ents) { or_entry_free(&e); st = OR_PANIC_INDEX_GAP; out->detail = (int64_t)k; goto fail; }
        for (int64_t j = (int64_t)k; j < n_ents; j++) or_entry_free(&ents[j]);
        n_ents = (int64_t)k;
        if (n_ents == cap_ents) { cap_ents = cap_ents ? cap_ents * 2 : 64; ents = (or_entry *)realloc(ents, sizeof(or_entry) * (size_t)cap_ents); }
        ents[n_ents++] = e;
        enti = ents[n_ents - 1].index;
      } else {
        enti = e.index;
        or_entry_free(&e);
      }
      break;
    }
    case 3: { /* stateType */
      or_hardstate s; memset(&s, 0, sizeof(s));
      int s2 = or_hardstate_unmarshal(rec.data, rec.data_len, &s);
      if (s2) { or_hardstate_free(&s); st = panic_class(s2, OR_PANIC_STATE); goto fail; }
      or_hardstate_free(&state);   /* state = mustUnmarshalState(rec.Data): the last one wins */
      state = s; has_state = 1;
      break;
    }
    case 1: /* metadataType */
      if (metadata != NULL && (rec.data == NULL || mlen != rec.data_len || memcmp(metadata, rec.data, (size_t)mlen) != 0)) {
        st = OR_ERR_METADATA_CONFLICT; goto fail;
      }
      free(metadata); metadata = NULL; mlen = 0;
      bytes_append(&metadata, &mlen, rec.data, rec.data_len);
      break;
    case 4: { /* crcType */
      uint32_t crc = dec.crc;
      if (crc != 0 && rec.crc != crc) { st = OR_ERR_WAL_CRC; goto fail; }
      dec.crc = rec.crc;                                 /* decoder.updateCRC */
      break;
    }
    default:
      st = OR_ERR_UNEXPECTED_TYPE; out->detail = rec.type; goto fail;
    }
    nrec++;
  }
  if (st != OR_EOF) goto fail;
  if (enti < ri) { st = OR_ERR_INDEX_NOT_FOUND; goto fail2; }
  or_record_free(&rec);
  out->status = OR_OK;
  out->n_records = nrec;
  out->last_crc = dec.crc;
  out->enti = enti;
  out->metadata = metadata; out->metadata_len = mlen;
  out->state = state; out->has_state = has_state;
  out->ents = ents; out->n_ents = n_ents;
  return OR_OK;
fail:
  out->fail_record = nrec;
  out->fail_offset = frame_off;
fail2:
  out->n_records = nrec;
  out->status = st;
  out->enti = enti;
  or_record_free(&rec);
  free(metadata);
  or_hardstate_free(&state);
  for (int64_t j = 0; j < n_ents; j++) or_entry_free(&ents[j]);
  free(ents);
  return st;
}

void or_readall_free(or_readall_result *r) {
  free(r->metadata);
  or_hardstate_free(&r->state);
  for (int64_t j = 0; j < r->n_ents; j++) or_entry_free(&r->ents[j]);
  free(r->ents);
  memset(r, 0, sizeof(*r));
}

int64_t or_chain_crcs(const uint8_t *buf, int64_t len, uint32_t *out, int64_t cap, int64_t *offsets) {
  or_decoder dec; or_decoder_init(&dec, buf, len);
  or_record rec; memset(&rec, 0, sizeof(rec));
  int64_t n = 0;
  for (;;) {
    int64_t off = dec.pos;
    int st = or_decode(&dec, &rec);
    if (st != OR_OK) break;
    if (rec.type == 4) {
      if (dec.crc != 0 && rec.crc != dec.crc) break;
      dec.crc = rec.crc;
    }
    if (n < cap) { out[n] = dec.crc; if (offsets) offsets[n] = off; }
    n++;
  }
  or_record_free(&rec);
  return n;
}

/* ===================================================================== */
/* encoder.encode (wal/encoder.go:25-37)                                  */
/* ===================================================================== */
void or_encoder_init(or_encoder *e, uint32_t prev_crc) {
  e->buf = NULL; e->len = 0; e->cap = 0; e->crc = prev_crc;
}
int or_encode(or_encoder *e, int64_t type, const uint8_t *data, int64_t n, int data_nil) {
  e->crc = or_crc32_update(e->crc, OR_CASTAGNOLI, data, (size_t)(data_nil ? 0 : n));
  int64_t sz = or_record_marshal(type, e->crc, data, n, data_nil, NULL);
  if (e->len + 8 + sz > e->cap) {
    int64_t nc = e->cap ? e->cap * 2 : 4096;
    while (nc < e->len + 8 + sz) nc *= 2;
    e->buf = (uint8_t *)realloc(e->buf, (size_t)nc); e->cap = nc;
  }
  memcpy(e->buf + e->len, &sz, 8);                      /* writeInt64, little endian */
  or_record_marshal(type, e->crc, data, n, data_nil, e->buf + e->len + 8);
  e->len += 8 + sz;
  return OR_OK;
}
void or_encoder_free(or_encoder *e) { free(e->buf); e->buf = NULL; e->len = e->cap = 0; }

/* ===================================================================== */
/* loadSnap (snap/snapshotter.go:76-111)                                  */
/* ===================================================================== */
int or_loadsnap(const uint8_t *file, int64_t len, uint32_t poly, or_loadsnap_result *out) {
  memset(out, 0, sizeof(*out));
  or_snappb s; memset(&s, 0, sizeof(s));
  int st = or_snappb_unmarshal(file, len, &s);
  if (st) { or_snappb_free(&s); return out->status = st; }
  out->stored_crc = s.crc;
  out->computed_crc = or_crc32_update(0, poly, s.data, (size_t)s.data_len);
  if (out->computed_crc != s.crc) { or_snappb_free(&s); return out->status = OR_ERR_SNAP_CRC; }
  st = or_snapshot_unmarshal(s.data, s.data_len, &out->snap);
  or_snappb_free(&s);
  if (st) { or_snapshot_free(&out->snap); return out->status = st; }
  return out->status = OR_OK;
}
void or_loadsnap_free(or_loadsnap_result *r) { or_snapshot_free(&r->snap); }

/* ===================================================================== */
/* raft.maybeCommit + raftLog.maybeCommit                                 */
/* ===================================================================== */
int or_maybe_commit(const uint64_t *match, int n, uint64_t term, uint64_t *committed,
                    const uint64_t *log_terms, uint64_t n_log, uint64_t offset) {
  if (n <= 0) return -OR_PANIC_BOUNDS;                  /* mis[q-1] on an empty slice */
  uint64_t mis[64];
  uint64_t *m = n <= 64 ? mis : (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
  memcpy(m, match, sizeof(uint64_t) * (size_t)n);
  /* sort.Sort(sort.Reverse(mis)) -- any correct sort gives the same order statistic */
  for (int i = 1; i < n; i++) {
    uint64_t v = m[i]; int j = i - 1;
    while (j >= 0 && m[j] < v) { m[j + 1] = m[j]; j--; }
    m[j + 1] = v;
  }
  int q = n / 2 + 1;
  uint64_t mci = m[q - 1];
  if (m != mis) free(m);
  if (!(mci > *committed)) return 0;
  uint64_t last = n_log - 1 + offset;                   /* lastIndex (uint64 wrap) */
  uint64_t t;
  if (mci < offset || mci > last) t = 0;                /* isOutOfBounds -> term 0 */
  else {
    uint64_t k = mci - offset;
    if (k >= n_log) return -OR_PANIC_BOUNDS;            /* &l.ents[i-l.offset] */
    t = log_terms[k];
  }
  if (t == term) { *committed = mci; return 1; }
  return 0;
}

/* The same rule over G groups in the GPU API's SoA layout (match[v*G + g],
 * log terms CSR) -- the CPU baseline of configs[4]; one call, no per-group
 * FFI cost.  status[g] = 0 or OR_PANIC_BOUNDS. */
void or_maybe_commit_batch(uint64_t G, const uint64_t *match, const uint8_t *nvoters, const uint64_t *term,
                           uint64_t *committed, const uint64_t *log_offset, const uint64_t *log_ptr,
                           const uint64_t *log_terms, uint8_t *changed, uint8_t *status) {
  for (uint64_t g = 0; g < G; g++) {
    uint64_t m[256];
    int n = nvoters[g];
    changed[g] = 0;
    status[g] = 0;
    /* no voters: mis[q-1] on an empty slice panics (raft/raft.go:255) */
    if (n <= 0) { status[g] = OR_PANIC_BOUNDS; continue; }
    for (int v = 0; v < n; v++) m[v] = match[(uint64_t)v * G + g];
    int rc = or_maybe_commit(m, n, term[g], &committed[g], log_terms + log_ptr[g], log_ptr[g + 1] - log_ptr[g],
                             log_offset[g]);
    if (rc < 0) status[g] = (uint8_t)(-rc);
    else changed[g] = (uint8_t)rc;
  }
}

/* raftpb.Message.MarshalTo, raft/raftpb/raft.pb.go:1010-1068 */
int64_t or_message_marshal(uint64_t type, uint64_t to, uint64_t from, uint64_t term, uint64_t log_term,
                           uint64_t index, const uint8_t *ents, const int64_t *ent_lens, int64_t n_ents,
                           uint64_t commit, const uint8_t *snap, int64_t snap_len, int reject, uint8_t *out) {
  int64_t i = 0, o = 0;
  i = put_byte(out, i, 0x08); i = put_varint(out, i, type);
  i = put_byte(out, i, 0x10); i = put_varint(out, i, to);
  i = put_byte(out, i, 0x18); i = put_varint(out, i, from);
  i = put_byte(out, i, 0x20); i = put_varint(out, i, term);
  i = put_byte(out, i, 0x28); i = put_varint(out, i, log_term);
  i = put_byte(out, i, 0x30); i = put_varint(out, i, index);
  for (int64_t k = 0; k < n_ents; k++) {
    i = put_byte(out, i, 0x3a); i = put_varint(out, i, (uint64_t)ent_lens[k]);
    i = put_bytes(out, i, ents + o, ent_lens[k]);
    o += ent_lens[k];
  }
  i = put_byte(out, i, 0x40); i = put_varint(out, i, commit);
  i = put_byte(out, i, 0x4a); i = put_varint(out, i, (uint64_t)snap_len); i = put_bytes(out, i, snap, snap_len);
  i = put_byte(out, i, 0x50); i = put_byte(out, i, reject ? 1 : 0);
  return i;
}


/* ---- checker helpers (test infrastructure, not restatements) ----------- */
/* A digest of ReadAll's ents for large parity cases: CRC-32C over every
 * entry's (type, term, index, nil flag, len, Data) in order. */
static uint32_t ents_digest_step(uint32_t h, int32_t type, uint64_t term, uint64_t index, int nil,
                                 const uint8_t *data, uint64_t n) {
  uint8_t hd[8 + 8 + 4 + 4 + 8];
  memcpy(hd, &term, 8);
  memcpy(hd + 8, &index, 8);
  memcpy(hd + 16, &type, 4);
  int32_t z = nil;
  memcpy(hd + 20, &z, 4);
  memcpy(hd + 24, &n, 8);
  h = or_crc32_update(h, OR_CASTAGNOLI, hd, sizeof(hd));
  return n ? or_crc32_update(h, OR_CASTAGNOLI, data, n) : h;
}

uint32_t or_ents_digest(const or_readall_result *r) {
  uint32_t h = 0;
  for (int64_t i = 0; i < r->n_ents; i++) {
    const or_entry *e = &r->ents[i];
    h = ents_digest_step(h, e->type, e->term, e->index, e->data == NULL, e->data, (uint64_t)e->data_len);
  }
  return h;
}

uint32_t or_ent_views_digest(const uint8_t *buf, const or_ent_view *v, int64_t n) {
  uint32_t h = 0;
  for (int64_t i = 0; i < n; i++)
    h = ents_digest_step(h, v[i].type, v[i].term, v[i].index, v[i].data_nil != 0, buf + v[i].data_off, v[i].data_len);
  return h;
}
