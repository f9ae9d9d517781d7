// ewal_device.h -- device-side building blocks shared by the WAL, snapshot and
// commit kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#define EW_PIECE 64                      // bytes per lane in the stream pass
#define EW_WAVE_BYTES 4096               // 64 lanes x 64 B
#define EW_WAVES 12                      // k_stream waves per workgroup (768 threads, 3 per SIMD)
#define EW_THREADS (EW_WAVES * 64)
#define EW_NIL 0xFFFFFFFFu
#define EW_SLOTS 32                      // candidate slots per 4 KiB unit
#define EW_VLOG 8                        // v[] holds lin of every 2^EW_VLOG = 256-B super-piece
#define EW_VPIECE (1 << EW_VLOG)
#define EW_VPU (EW_WAVE_BYTES / EW_VPIECE)  // v[] values per 4 KiB unit (16)

// ---- shift operators S_{2^m} -------------------------------------------
// Byte tables: tb[k*256 + b] = S_{2^m}(b << 8k).
__device__ __forceinline__ uint32_t tab_apply(const uint32_t *tb, uint32_t x) {
  return tb[x & 0xff] ^ tb[256 + ((x >> 8) & 0xff)] ^ tb[512 + ((x >> 16) & 0xff)] ^ tb[768 + (x >> 24)];
}
// global tables, m = 0..47
__device__ __forceinline__ uint32_t gshift_pow2(const uint32_t *g, int m, uint32_t x) {
  return tab_apply(g + (size_t)m * 1024, x);
}
__device__ __forceinline__ uint32_t gshift_n(const uint32_t *g, uint64_t n, uint32_t x) {
  while (n) {
    int m = __builtin_ctzll(n);
    n &= n - 1;
    x = gshift_pow2(g, m, x);
  }
  return x;
}

// A shift operator as eight nibble tables (t[k * 16 + d] = S(d << 4k)): 8
// lookups per application, 512 B of LDS per operator.
__device__ __forceinline__ uint32_t nib_apply(const uint32_t *t, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r ^= t[k * 16 + ((x >> (4 * k)) & 15)];
  return r;
}

// Copy n dwords into LDS: dst[i] = src(i).  Every thread issues 16 loads
// before its first store (a plain strided copy loop waits on each load in
// turn, one L2 round trip per iteration).  Indices past n load a clamped
// address and are not stored.
template <int NT, class F>
__device__ __forceinline__ void stage_lds(uint32_t *dst, int n, F src) {
  const int tid = threadIdx.x;
  for (int i0 = 0; i0 < n; i0 += 16 * NT) {
    uint32_t r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = i0 + k * NT + tid;
      r[k] = src(i < n ? i : n - 1);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = i0 + k * NT + tid;
      if (i < n) dst[i] = r[k];
    }
  }
}

// Slicing-by-4 step on a register already XORed with the next data word;
// tables t[4][256] (t[0] = MakeTable(poly)), non-replicated layout.
__device__ __forceinline__ uint32_t step4_flat(const uint32_t *t, uint32_t c) {
  return t[768 + (c & 0xff)] ^ t[512 + ((c >> 8) & 0xff)] ^ t[256 + ((c >> 16) & 0xff)] ^ t[c >> 24];
}
// raw register continue over bytes [o, e) of buf (plain global loads).
__device__ __forceinline__ uint32_t raw_bytes(const uint32_t *t, uint32_t c, const uint8_t *buf, uint64_t o, uint64_t e) {
  while (o < e && (o & 3)) { c = t[(c ^ buf[o]) & 0xff] ^ (c >> 8); ++o; }
  while (o + 4 <= e) { c = step4_flat(t, c ^ *(const uint32_t *)(buf + o)); o += 4; }
  while (o < e) { c = t[(c ^ buf[o]) & 0xff] ^ (c >> 8); ++o; }
  return c;
}

// ---- byte sources for the protobuf walkers --------------------------------
// A plain global pointer, or WinReader: the first n bytes from an LDS copy
// (the frame head k_decode loaded with a few vector loads), the rest from
// global memory.  gptr() is the global address of byte 0 (proto.Skip).
struct WinReader {
  const uint8_t *w;   // LDS copy of bytes [0, n)
  int64_t n;
  const uint8_t *g;   // the same bytes in global memory
  __device__ __forceinline__ uint8_t operator[](int64_t i) const { return i < n ? w[i] : g[i]; }
};
__device__ __forceinline__ WinReader operator+(const WinReader &r, int64_t k) {
  return WinReader{r.w + k, r.n - k, r.g + k};
}
__device__ __forceinline__ const uint8_t *gptr(const uint8_t *p) { return p; }
__device__ __forceinline__ const uint8_t *gptr(const WinReader &r) { return r.g; }

// ---- Go varint readers (shifts >= width give 0) --------------------------
// Reads buf[base+i...] while i < l; returns 0 or EWAL_ERR_UNEXPECTED_EOF (2).
// width 32 keeps Go's uint32/int32 truncation ((uint32(b)&0x7F) << 28 loses bits).
template <class P>
__device__ __forceinline__ int rd_varint(const P &p, int64_t &i, int64_t l, uint64_t &v, int width) {
  for (uint32_t shift = 0;; shift += 7) {
    if (i >= l) return 2;
    uint8_t b = p[i++];
    if (shift < (uint32_t)width) v |= (uint64_t)(b & 0x7F) << shift;
    if (width == 32) v &= 0xffffffffull;
    if (b < 0x80) return 0;
  }
}

// ---- proto.Skip (third_party/code.google.com/p/gogoprotobuf/proto/skip_gogo.go:33-116)
// Iterative restatement of the group recursion with a bounded frame stack.
// Exact non-termination tests: a frame looping more times than it has byte
// positions must revisit one (deterministic => forever), and a child group
// pushed at local start 0 re-enters its parent (infinite recursion) -> 37.
#define PB_SKIP_DEPTH 16
__device__ __forceinline__ int skip_wire(const uint8_t *p, int64_t &i, int64_t l, uint64_t &w) {
  w = 0;
  for (uint32_t shift = 0;; shift += 7) {
    if (i >= l) return 2;       // io.ErrUnexpectedEOF
    if (i < 0) return 33;       // data[index] with index < 0: runtime panic
    uint8_t b = p[i++];
    if (shift < 64) w |= (uint64_t)(b & 0x7F) << shift;
    if (b < 0x80) return 0;
  }
}
__device__ __forceinline__ int skip_simple(const uint8_t *p, int64_t l, int wt, int64_t i, int64_t &n) {
  switch (wt) {
  case 0:
    for (;;) {
      if (i >= l) return 2;
      ++i;
      if (p[i - 1] < 0x80) break;
    }
    n = i;
    return 0;
  case 1: n = (int64_t)((uint64_t)i + 8); return 0;
  case 2: {
    uint64_t len = 0;
    for (uint32_t shift = 0;; shift += 7) {
      if (i >= l) return 2;
      uint8_t b = p[i++];
      if (shift < 64) len |= (uint64_t)(b & 0x7F) << shift;
      if (b < 0x80) break;
    }
    n = (int64_t)((uint64_t)i + len);
    return 0;
  }
  case 4: n = i; return 0;
  case 5: n = (int64_t)((uint64_t)i + 4); return 0;
  default: return 7;            // proto.ErrWrongType
  }
}
__device__ __noinline__ int pb_skip(const uint8_t *p, int64_t l, int64_t &out) {
  if (l <= 0) return 33;        // panic("unreachable")
  int64_t i = 0;
  uint64_t w;
  int st = skip_wire(p, i, l, w);
  if (st) return st;
  int wt = (int)(w & 7);
  if (wt != 3) return skip_simple(p, l, wt, i, out);
  int64_t sb[PB_SKIP_DEPTH], ss[PB_SKIP_DEPTH], si[PB_SKIP_DEPTH];
  int depth = 0;
  int64_t base = 0, idx = i, iters = 0;
  for (;;) {
    const uint8_t *d = p + base;
    const int64_t ll = l - base;
    if (++iters > ll + 1) return 37;
    const int64_t start = idx;
    int64_t j = idx;
    st = skip_wire(d, j, ll, w);
    if (st) return st;
    const int wt2 = (int)(w & 7);
    if (wt2 == 4) {
      if (depth == 0) { out = j; return 0; }
      --depth;
      base = sb[depth];
      idx = (int64_t)((uint64_t)ss[depth] + (uint64_t)j);
      iters = si[depth];
      continue;
    }
    if (wt2 == 3) {
      if (start == 0) return 37;
      if (depth == PB_SKIP_DEPTH) return 48;
      sb[depth] = base; ss[depth] = start; si[depth] = iters;
      ++depth;
      base += start;
      idx = j - start;
      iters = 0;
      continue;
    }
    int64_t nn;
    st = skip_simple(d + start, ll - start, wt2, j - start, nn);
    if (st) return st;
    idx = (int64_t)((uint64_t)start + (uint64_t)nn);
  }
}

// ---- gogoprotobuf Unmarshal walker (exact Go semantics on the supported set)
// Field kinds are compile-time template arguments (no runtime-indexed state,
// so nothing spills to scratch): PB_NONE (unknown -> proto.Skip into
// XXX_unrecognized, sets unrec), PB_VAR64/PB_VAR32 (|= accumulate), PB_BYTES
// (append; nil when empty), PB_REP64 (append to a repeated list in rep[]).
// Returns 0, 2 (io.ErrUnexpectedEOF), 7 (proto.ErrWrongType), 33 (bounds
// panic), 37 (never terminates) or 48 (EWAL_UNSUPPORTED_ENCODING: group
// nesting deeper than the device stack).  The walk always runs to Go's own
// result: a bytes field whose repeats concatenate non-empty segments (Go's
// `m.Data = append(m.Data, ...)`) or a repeated list longer than rep's
// capacity only sets the field's `split` flag (boff = the first segment,
// blen = the total length), for the caller to decide.
#define PB_NONE 0
#define PB_VAR64 1
#define PB_VAR32 2
#define PB_BYTES 3
#define PB_REP64 4
struct PbField {
  uint64_t v;      // varint value (OR-accumulated) / repeated count
  int64_t boff;    // bytes field offset (-1: nil)
  int64_t blen;
  uint32_t split;  // bytes: more than one non-empty segment; repeated: past rep's capacity
};
__device__ __forceinline__ void pbf_init(PbField &f) { f.v = 0; f.boff = -1; f.blen = 0; f.split = 0; }

template <int K, class P>
__device__ __forceinline__ int pb_field(const P &p, int64_t &i, int64_t l, int wt, PbField &f, uint64_t *rep,
                                        uint32_t repcap) {
  if (K == PB_BYTES) {
    if (wt != 2) return 7;
    uint64_t bl = 0;
    if (rd_varint(p, i, l, bl, 64)) return 2;
    int64_t post = (int64_t)((uint64_t)i + bl);
    if (post > l) return 2;
    if (post < i) return 33;
    if (post > i) {
      if (f.blen > 0) {
        f.split = 1;
        f.blen += post - i;
      } else {
        f.boff = i;
        f.blen = post - i;
      }
    }
    i = post;
    return 0;
  } else if (K == PB_REP64) {
    if (wt != 0) return 7;
    uint64_t v = 0;
    if (rd_varint(p, i, l, v, 64)) return 2;
    if (f.v >= repcap) f.split = 1;
    else if (rep) rep[f.v] = v;
    f.v++;
    return 0;
  } else {
    if (wt != 0) return 7;
    return rd_varint(p, i, l, f.v, K == PB_VAR32 ? 32 : 64) ? 2 : 0;
  }
}

// unk(i, hi): every unknown field [i, hi) the walk appends to XXX_unrecognized
struct PbNoUnk {
  __device__ void operator()(int64_t, int64_t) const {}
};
template <int K1, int K2, int K3, int K4, int K5, class P, class U = PbNoUnk>
__device__ inline int pb_walk(const P &p, int64_t l, PbField &f1, PbField &f2, PbField &f3, PbField &f4,
                              PbField &f5, int &unrec, uint64_t *rep2, uint64_t *rep5, uint32_t repcap,
                              U unk = U()) {
  int64_t i = 0;
  unrec = 0;
  while (i < l) {
    uint64_t wire = 0;
    if (rd_varint(p, i, l, wire, 64)) return 2;
    const uint32_t fn = (uint32_t)(wire >> 3);   // int32(wire >> 3)
    const int wt = (int)(wire & 7);
    int st = -1;
    switch (fn) {
    case 1: if (K1 != PB_NONE) st = pb_field<K1>(p, i, l, wt, f1, nullptr, 0); break;
    case 2: if (K2 != PB_NONE) st = pb_field<K2>(p, i, l, wt, f2, rep2, repcap); break;
    case 3: if (K3 != PB_NONE) st = pb_field<K3>(p, i, l, wt, f3, nullptr, 0); break;
    case 4: if (K4 != PB_NONE) st = pb_field<K4>(p, i, l, wt, f4, nullptr, 0); break;
    case 5: if (K5 != PB_NONE) st = pb_field<K5>(p, i, l, wt, f5, rep5, repcap); break;
    default: break;
    }
    if (st > 0) return st;
    if (st == 0) continue;
    // default: index -= sizeOfWire; Skip(data[index:]); bounds; append
    int64_t sow = 0;
    uint64_t w = wire;
    do { ++sow; w >>= 7; } while (w);
    i -= sow;
    int64_t skippy;
    st = pb_skip(gptr(p) + i, l - i, skippy);
    if (st) return st;
    int64_t hi = (int64_t)((uint64_t)i + (uint64_t)skippy);
    if (hi > l) return 2;
    if (hi < i) return 33;
    if (skippy == 0) return 37;
    unrec = 1;
    unk(i, hi);
    i = hi;
  }
  return 0;
}

// Every occurrence of field fnum that pb_walk consumed over the same bytes,
// in order: f(true, off, len) for a non-empty bytes occurrence, f(false,
// value, 0) for a varint one.  Other fields are stepped over by proto.Skip
// from their tag; kvar / kbytes (bit fn) name the message's varint / bytes
// fields, so a known field with the wrong wire type ends the walk where
// Unmarshal's ErrWrongType does (a message whose error is discarded keeps
// what came before it).
template <class F>
__device__ void pb_each(const uint8_t *p, int64_t l, uint32_t fnum, uint32_t kvar, uint32_t kbytes, F f) {
  int64_t i = 0;
  while (i < l) {
    const int64_t tag = i;
    uint64_t wire = 0;
    if (rd_varint(p, i, l, wire, 64)) return;
    const uint32_t fn = (uint32_t)(wire >> 3);
    const int wt = (int)(wire & 7);
    if (fn < 32 && ((((kvar >> fn) & 1) && wt != 0) || (((kbytes >> fn) & 1) && wt != 2))) return;
    if (fn == fnum && wt == 0) {
      uint64_t v = 0;
      if (rd_varint(p, i, l, v, 64)) return;
      f(false, v, 0ull);
      continue;
    }
    if (fn == fnum && wt == 2) {
      uint64_t bl = 0;
      if (rd_varint(p, i, l, bl, 64)) return;
      const int64_t post = (int64_t)((uint64_t)i + bl);
      if (post > l || post < i) return;
      if (post > i) f(true, (uint64_t)i, (uint64_t)(post - i));
      i = post;
      continue;
    }
    int64_t sk;
    if (pb_skip(p + tag, l - tag, sk) || sk <= 0) return;
    i = tag + sk;
  }
}
