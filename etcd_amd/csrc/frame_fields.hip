// frame_fields.hip -- the per-frame helpers the frame pass (frame_kernels.hip)
// shares with its result gathers: the canonical field parse of one frame
// re-read from global memory (fc_frame_fields), the single-frame CRC verdict
// (fc_check_one), the nibble-table source layout (nib_src) and the
// nontemporal ents store.
//
// Reference: decoder.decode wal/decoder.go:28-47, walpb.Record.Unmarshal
// wal/walpb/record.pb.go:43-136, raftpb.Entry / HardState.Unmarshal
// raft/raftpb/raft.pb.go:170-277, 618-704.
#include "ewal_device.h"
#include "ewal_internal.h"

// The single WAL's ents are written with nontemporal stores (40 B per op,
// read back only by the host's copy or the next call): configs[1]
// post-stream -8 us; the batched path keeps plain stores (+1-2 % with
// nontemporal ones, profiles/r02/ab_nt_ents.txt).
// the same with relaxed agent-scope atomic stores (sc1: the lines leave L2; A/B EW_ENTS_SC1)
__device__ __forceinline__ void store_entry_sc1(ewal_entry *dst, const ewal_entry &e) {
  uint64_t *q = (uint64_t *)dst;
  __hip_atomic_store(q, e.term, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, e.index, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 2, e.data_off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 3, e.data_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 4, ((uint64_t)(uint32_t)e.data_nil << 32) | (uint32_t)e.type, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_entry_nt(ewal_entry *dst, const ewal_entry &e) {
  uint64_t *q = (uint64_t *)dst;
  __builtin_nontemporal_store(e.term, q);
  __builtin_nontemporal_store(e.index, q + 1);
  __builtin_nontemporal_store(e.data_off, q + 2);
  __builtin_nontemporal_store(e.data_len, q + 3);
  __builtin_nontemporal_store(((uint64_t)(uint32_t)e.data_nil << 32) | (uint32_t)e.type, q + 4);
}

// decoder.decode's check + ReadAll's crc-record rule for one frame (k_check's
// per-frame verdict): *chained = the running CRC after it.
__device__ __forceinline__ int fc_check_one(const uint32_t *g_shift, int32_t type, uint32_t crc, uint32_t seed,
                                            uint32_t pfd, uint32_t pe, uint64_t dlen, uint32_t *chained) {
  if (type == 4) {
    *chained = crc;
    return (seed != 0 && crc != seed) ? EWAL_ERR_WAL_CRC : 0;
  }
  uint32_t computed = seed;
  if (dlen) computed = gshift_n(g_shift, dlen, seed ^ 0xffffffffu ^ pfd) ^ pe ^ 0xffffffffu;
  *chained = computed;
  if (computed != crc) return EWAL_ERR_RECORD_CRC;
  return (type != 1 && type != 2 && type != 3) ? EWAL_ERR_UNEXPECTED_TYPE : 0;
}

// S_{2^m} as nibble tables: N[m][k][d] = S_{2^m}(d << 4k), 8 x 16 entries per
// operator (512 B instead of a 4 KiB byte table), 8 lookups per application.
__device__ __forceinline__ uint32_t nib_src(const uint32_t *g_shift, int i) {
  const int m = i >> 7, k = (i >> 4) & 7, d = i & 15;
  return g_shift[m * 1024 + (k >> 1) * 256 + (d << (4 * (k & 1)))];
}

// The canonical layout etcd's encoder writes (record.pb.go:175-196,
// raft.pb.go:921-943, 1079-1097): every field once, in order, the last one
// ending at the message end -- parsed straight from the frame's head bytes
// h[0..n) (n >= 81: every canonical head fits).  false: not canonical.
__device__ __forceinline__ bool fc_varint(const uint8_t *h, int n, int &o, uint64_t &v) {
  uint64_t x = 0;
  for (int s = 0; s < 64 && o < n; s += 7) {
    const uint8_t b = h[o++];
    x |= (uint64_t)(b & 0x7f) << s;
    if (b < 0x80) { v = x; return true; }
  }
  return false;
}
__device__ __forceinline__ bool fc_tag_varint(const uint8_t *h, int n, int &o, uint8_t tag, uint64_t &v) {
  return o < n && h[o++] == tag && fc_varint(h, n, o, v);
}
__device__ bool fc_canon_fields(const uint8_t *h, int n, uint64_t p, int64_t L, RecDesc &d) {
  int o = 8;
  uint64_t ty, cr, dl = 0;
  if (!fc_tag_varint(h, n, o, 0x08, ty) || !fc_tag_varint(h, n, o, 0x10, cr)) return false;
  const bool hasd = (int64_t)(o - 8) < L;
  if (hasd && !fc_tag_varint(h, n, o, 0x1a, dl)) return false;
  if ((int64_t)(o - 8) + (int64_t)dl != L) return false;
  d.type = (int64_t)ty;
  d.crc = (uint32_t)cr;
  if (dl > 0) { d.doff = p + (uint64_t)o; d.dlen = dl; d.dnil = 0; }
  if (dl == 0 || (d.type != 2 && d.type != 3)) return true;
  const int e0 = o;
  uint64_t f0, f1, f2;
  if (!fc_tag_varint(h, n, o, 0x08, f0) || !fc_tag_varint(h, n, o, 0x10, f1) || !fc_tag_varint(h, n, o, 0x18, f2))
    return false;
  if (d.type == 3) {
    if ((uint64_t)(o - e0) != dl) return false;
    d.f0 = f0; d.f1 = f1; d.f2 = f2;
    return true;
  }
  uint64_t el = 0;
  const bool hase = (uint64_t)(o - e0) < dl;
  if (hase && !fc_tag_varint(h, n, o, 0x22, el)) return false;
  if ((uint64_t)(o - e0) + el != dl) return false;
  d.etype = (int32_t)(uint32_t)f0;
  d.f0 = f1;
  d.f1 = f2;
  if (el > 0) { d.edoff = p + (uint64_t)o; d.edlen = el; d.enil = 0; }
  return true;
}

// Every field a later pass needs of one canonical frame, re-read from global
// memory (the passes after the frame pass touch a handful of frames): Record type /
// crc / Data, Entry / HardState fields.  The first 96 bytes come in with six
// vector loads into this thread's LDS slot w (96 B), the walkers read the
// rest (if any) from global memory.
__device__ RecDesc fc_frame_fields(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p, uint4 *w) {
  RecDesc d;
  d.off = p;
  d.type = 0; d.crc = 0; d.chained = 0; d.st = 0; d.sub_st = 0;
  d.doff = p + 8; d.dlen = 0; d.dnil = 1;
  d.f0 = d.f1 = d.f2 = 0; d.edoff = 0; d.edlen = 0; d.enil = 1; d.etype = 0; d.pad0 = 0; d.pad1 = 0;
  if (p + 8 > B) {   // not a frame (only a void pass asks)
    d.st = EWAL_ERR_UNEXPECTED_EOF;
    return d;
  }
  // the 96 bytes from the 16-B boundary below p in one round trip; the
  // length prefix is read back from them (p - p16 + 8 <= 24)
  const uint64_t p16 = p & ~15ull;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint64_t o = p16 + 16 * k;
    uint4 x;
    if (o + 16 <= B) {
      x = *(const uint4 *)(buf + o);
    } else {
      uint32_t y[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = load_word_guarded(buf, B, o + 4 * j);
      x = make_uint4(y[0], y[1], y[2], y[3]);
    }
    w[k] = x;
  }
  int64_t L = 0;
  {
    const uint8_t *hb = (const uint8_t *)w + (p - p16);
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= (uint64_t)hb[i] << (8 * i);
    L = (int64_t)v;
  }
  if (L < 0 || (uint64_t)L > B - p - 8) {
    d.st = EWAL_ERR_UNEXPECTED_EOF;
    return d;
  }
  if (fc_canon_fields((const uint8_t *)w + (p - p16), 96 - (int)(p - p16), p, L, d)) return d;
  // not the canonical layout (a frame the general path also decodes): the walkers
  const WinReader R0{(const uint8_t *)w + (p - p16), (int64_t)(96 - (p - p16)), buf + p};
  const WinReader rb = R0 + 8;
  PbField a1, a2, a3, a4, a5;
  pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
  int unrec = 0;
  d.st = pb_walk<PB_VAR64, PB_VAR32, PB_BYTES, PB_NONE, PB_NONE>(rb, L, a1, a2, a3, a4, a5, unrec, nullptr, nullptr, 0);
  d.type = (int64_t)a1.v;
  d.crc = (uint32_t)a2.v;
  if (a3.blen > 0) { d.doff = p + 8 + (uint64_t)a3.boff; d.dlen = (uint64_t)a3.blen; d.dnil = 0; }
  if (d.st == 0 && d.dlen && (d.type == 2 || d.type == 3)) {
    const WinReader dp = R0 + (int64_t)(d.doff - p);
    PbField e1, e2, e3, e4, e5;
    pbf_init(e1); pbf_init(e2); pbf_init(e3); pbf_init(e4); pbf_init(e5);
    int ur = 0;
    if (d.type == 2) {
      d.sub_st = pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(dp, (int64_t)d.dlen, e1, e2, e3, e4, e5, ur,
                                                                          nullptr, nullptr, 0);
      d.etype = (int32_t)(uint32_t)e1.v;
      d.f0 = e2.v;
      d.f1 = e3.v;
      if (e4.blen > 0) { d.edoff = d.doff + (uint64_t)e4.boff; d.edlen = (uint64_t)e4.blen; d.enil = 0; }
    } else {
      d.sub_st = pb_walk<PB_VAR64, PB_VAR64, PB_VAR64, PB_NONE, PB_NONE>(dp, (int64_t)d.dlen, e1, e2, e3, e4, e5, ur,
                                                                         nullptr, nullptr, 0);
      d.f0 = e1.v; d.f1 = e2.v; d.f2 = e3.v;
    }
  }
  return d;
}
