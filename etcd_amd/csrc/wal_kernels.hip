// wal_kernels.hip -- the WAL replay-and-verify pipeline for gfx950.
//
// Reference path (mzsanford/etcd v0.5.0-alpha):
//   wal/wal.go:164-216  (*WAL).ReadAll      -- dispatch, chain re-seed, ents
//   wal/decoder.go:28-47 decoder.decode     -- int64 length framing + Unmarshal + CRC
//   wal/walpb/record.pb.go:43-136           -- Record.Unmarshal
//   pkg/crc/crc.go:23-41 + hash/crc32       -- chained CRC-32C
//   raft/raftpb/raft.pb.go:170-277,618-704  -- Entry / HardState Unmarshal
//
// Kernels (one HBM pass over the WAL bytes, then per-frame work):
//   k_stream   fused: per-lane CRC (slicing-by-4, LDS tables), frame-start
//              candidate detection, wave/tile affine CRC reduction and the
//              device-wide decoupled look-back that turns tile CRCs into
//              stream prefixes P(x) = lin(stream[0..x)) at every 4 KiB, plus
//              the ordered candidate list.
//   k_link     candidate -> successor candidate (pos + 8 + len).
//   k_runs / k_jump / k_mark / k_entry / k_member
//              framing: the true frame chain from byte 0 by pointer jumping
//              over runs of consecutive candidates.
//   k_decode   walpb.Record / raftpb.Entry / HardState decode per frame.
//   k_verify   chained CRC check per frame against its predecessor's stored
//              CRC (== the reference's running CRC up to the first failure),
//              using the stream prefixes: Update(seed, D[s,e)) =
//              S_n(seed ^ ~0 ^ P(s)) ^ P(e) ^ ~0.
//   k_meta / k_ops / k_gap / k_ents: ReadAll's metadata / ents semantics.
#include "ewal_device.h"
#include "ewal_internal.h"

// ===========================================================================
// k_stream
// ===========================================================================
__device__ __forceinline__ uint32_t lds_step4(const uint32_t *s, int cl, uint32_t c) {
  // s[(t*256 + b) * EW_R + cl]
  return s[((3 * 256 + (c & 0xff)) * EW_R) + cl] ^ s[((2 * 256 + ((c >> 8) & 0xff)) * EW_R) + cl] ^
         s[((1 * 256 + ((c >> 16) & 0xff)) * EW_R) + cl] ^ s[((0 * 256 + (c >> 24)) * EW_R) + cl];
}
__device__ __forceinline__ uint32_t lds_shift(const uint32_t *s, int m, uint32_t x) {
  return tab_apply(s + (m - EW_LDS_SHIFT0) * 1024, x);
}

__device__ __forceinline__ uint32_t load_word_guarded(const uint8_t *buf, uint64_t B, uint64_t o) {
  if (o + 4 <= B) return *(const uint32_t *)(buf + o);
  uint32_t w = 0;
  for (int i = 0; i < 4; ++i)
    if (o + i < B) w |= (uint32_t)buf[o + i] << (8 * i);
  return w;
}

// Exact frame-start test at lane-local byte o = 4*j + k.  D holds the lane's
// 16 dwords plus the next 3.  A candidate has int64 length L in [4, B-p-8]
// and the canonical Record head 08 <type<0x80> 10 (record.pb.go:175-196).
#define CAND_TEST(J)                                                                 \
  {                                                                                  \
    uint32_t x_ = D[(J) + 2];                                                        \
    uint32_t y_ = __builtin_amdgcn_alignbyte(D[(J) + 3], D[(J) + 2], 2);             \
    uint32_t z_ = (x_ ^ 0x08080808u) | (y_ ^ 0x10101010u);                           \
    uint32_t m_ = (z_ - 0x01010101u) & ~z_ & 0x80808080u;                            \
    while (m_) {                                                                     \
      uint32_t k_ = (uint32_t)__builtin_ctz(m_) >> 3;                                \
      m_ &= m_ - 1;                                                                  \
      uint32_t lo_ = __builtin_amdgcn_alignbyte(D[(J) + 1], D[(J)], k_);             \
      uint32_t hi_ = __builtin_amdgcn_alignbyte(D[(J) + 2], D[(J) + 1], k_);         \
      uint32_t hd_ = __builtin_amdgcn_alignbyte(D[(J) + 3], D[(J) + 2], k_);         \
      uint64_t p_ = off + 4 * (J) + k_;                                              \
      uint64_t L_ = ((uint64_t)hi_ << 32) | lo_;                                     \
      bool ok_ = ((hd_ & 0xff) == 0x08) && (((hd_ >> 8) & 0xff) < 0x80) &&           \
                 (((hd_ >> 16) & 0xff) == 0x10) && ((int64_t)L_ >= 4) &&             \
                 (p_ + 8 <= B) && (L_ <= B - p_ - 8);                                \
      if (ok_) { CAND_ACTION; }                                                      \
    }                                                                                \
  }

__device__ __forceinline__ uint32_t count_cands(const uint32_t (&D)[19], uint64_t off, uint64_t B) {
  uint32_t cnt = 0;
#define CAND_ACTION ++cnt
  CAND_TEST(0) CAND_TEST(1) CAND_TEST(2) CAND_TEST(3) CAND_TEST(4) CAND_TEST(5) CAND_TEST(6) CAND_TEST(7)
  CAND_TEST(8) CAND_TEST(9) CAND_TEST(10) CAND_TEST(11) CAND_TEST(12) CAND_TEST(13) CAND_TEST(14) CAND_TEST(15)
#undef CAND_ACTION
  return cnt;
}

__device__ __forceinline__ void write_cands(const uint32_t (&D)[19], uint64_t off, uint64_t B, uint64_t base,
                                            uint64_t *cpos, uint64_t *clen, uint64_t ccap) {
  uint64_t w = base;
#define CAND_ACTION                      \
  if (w < ccap) { cpos[w] = p_; clen[w] = L_; } \
  ++w
  CAND_TEST(0) CAND_TEST(1) CAND_TEST(2) CAND_TEST(3) CAND_TEST(4) CAND_TEST(5) CAND_TEST(6) CAND_TEST(7)
  CAND_TEST(8) CAND_TEST(9) CAND_TEST(10) CAND_TEST(11) CAND_TEST(12) CAND_TEST(13) CAND_TEST(14) CAND_TEST(15)
#undef CAND_ACTION
}

// Decoupled look-back (Merrill & Garland) over 64 predecessors per step.
// Returns (X, N): the stream prefix lin(stream[0 .. t*TILE)) and the number
// of candidates before tile t; publishes tile t's inclusive values.
__device__ __forceinline__ void lookback(TileDesc *desc, uint32_t t, uint32_t agg, uint32_t cnt,
                                         const uint32_t *g_shift, uint32_t &X, unsigned long long &N,
                                         uint32_t *errflag) {
  const int lane = threadIdx.x & 63;
  uint32_t accx = 0;
  unsigned long long accn = 0;
  if (t > 0) {
    if (lane == 0) st_agent(&desc[t].agg, EW_DESC_VALID | ((unsigned long long)cnt << 32) | agg);
    uint64_t acc_tiles = 0;
    int64_t j = (int64_t)t - 1;
    uint32_t spins = 0;
    for (;;) {
      int64_t idx = j - lane;
      unsigned long long inc = 0, ag = 0;
      int st;
      if (idx < 0) {
        st = 2;
      } else {
        inc = ld_agent(&desc[idx].inc);
        if (inc & EW_DESC_VALID) {
          st = 2;
        } else {
          ag = ld_agent(&desc[idx].agg);
          st = (ag & EW_DESC_VALID) ? 1 : 0;
        }
      }
      unsigned long long m2 = __ballot(st == 2), m0 = __ballot(st == 0);
      int f2 = m2 ? __ffsll((long long)m2) - 1 : 64;
      int f0 = m0 ? __ffsll((long long)m0) - 1 : 64;
      if (f2 < f0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t term = 0;
        unsigned long long tn = 0;
        if (lane < f2) {
          term = gshift_n(g_shift, (acc_tiles + lane) << EW_TILE_LOG2, (uint32_t)ag);
          tn = (ag >> 32) & 0x7fffffffull;
        } else if (lane == f2 && idx >= 0) {
          tn = ld_agent(&desc[idx].inc_cnt);
          term = gshift_n(g_shift, (acc_tiles + lane) << EW_TILE_LOG2, (uint32_t)inc);
        }
        accx ^= wave_xor(term);
        accn += wave_sum64(tn);
        break;
      }
      if (f0 < 64) {
        if (++spins > (1u << 24)) {
          if (lane == 0) atomicOr(errflag, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint32_t term = gshift_n(g_shift, (acc_tiles + lane) << EW_TILE_LOG2, (uint32_t)ag);
      accx ^= wave_xor(term);
      accn += wave_sum64((ag >> 32) & 0x7fffffffull);
      acc_tiles += 64;
      j -= 64;
    }
  }
  X = accx;
  N = accn;
  if (lane == 0) {
    uint32_t I = gshift_pow2(g_shift, EW_TILE_LOG2, accx) ^ agg;
    st_agent(&desc[t].inc_cnt, accn + cnt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_agent(&desc[t].inc, EW_DESC_VALID | (unsigned long long)I);
  }
}

__global__ __launch_bounds__(EW_THREADS, 1) void k_stream(StreamArgs a) {
  __shared__ uint32_t s_slice[4 * 256 * EW_R];        // 64 KiB, replicated slicing tables
  __shared__ uint32_t s_shift[EW_LDS_SHIFTS * 1024];  // 40 KiB, S_{2^6}..S_{2^15}
  __shared__ uint32_t s_wagg[EW_WAVES];
  __shared__ uint32_t s_wcnt[EW_WAVES];
  __shared__ unsigned long long s_wbase[EW_WAVES];
  __shared__ uint32_t s_tile;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < 4 * 256 * EW_R; i += EW_THREADS) s_slice[i] = a.g_slice[i / EW_R];
  for (int i = tid; i < EW_LDS_SHIFTS * 1024; i += EW_THREADS) s_shift[i] = a.g_shift[EW_LDS_SHIFT0 * 1024 + i];
  const int cl = lane & (EW_R - 1);
  const uint64_t B = a.B;

  for (;;) {
    __syncthreads();
    if (tid == 0) s_tile = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const uint32_t t = s_tile;
    if (t >= a.ntiles) break;

    const uint64_t off = (uint64_t)t * EW_TILE + (uint64_t)wv * EW_WAVE_BYTES + (uint64_t)lane * EW_PIECE;
    uint32_t D[19];
    if (off + EW_PIECE <= B) {
      const uint4 *p = (const uint4 *)(a.buf + off);
      uint4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
      D[0] = q0.x; D[1] = q0.y; D[2] = q0.z; D[3] = q0.w;
      D[4] = q1.x; D[5] = q1.y; D[6] = q1.z; D[7] = q1.w;
      D[8] = q2.x; D[9] = q2.y; D[10] = q2.z; D[11] = q2.w;
      D[12] = q3.x; D[13] = q3.y; D[14] = q3.z; D[15] = q3.w;
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) D[k] = (off < B) ? load_word_guarded(a.buf, B, off + 4 * k) : 0u;
    }

    // lin(piece) with conflict-light replicated slicing tables
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) c = lds_step4(s_slice, cl, c ^ D[k]);
    a.v[(uint64_t)t * EW_THREADS + tid] = c;

    uint32_t cnt = 0;
    if (a.find_cand) {
      D[16] = __shfl_down(D[0], 1);
      D[17] = __shfl_down(D[1], 1);
      D[18] = __shfl_down(D[2], 1);
      if (lane == 63) {
        const uint64_t o = off + EW_PIECE;
        D[16] = load_word_guarded(a.buf, B, o);
        D[17] = load_word_guarded(a.buf, B, o + 4);
        D[18] = load_word_guarded(a.buf, B, o + 8);
      }
      if (off < B) cnt = count_cands(D, off, B);
    }

    // wave reduction of the affine CRC: lane 0 ends with lin(wave's 4 KiB)
    uint32_t r = c;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      uint32_t o = __shfl_down(r, 1 << d);
      if ((lane & ((2 << d) - 1)) == 0) r = lds_shift(s_shift, EW_LDS_SHIFT0 + d, r) ^ o;
    }
    // wave inclusive scan of candidate counts
    uint32_t ci = cnt;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      uint32_t o = __shfl_up(ci, 1 << d);
      if (lane >= (1 << d)) ci += o;
    }
    if (lane == 0) s_wagg[wv] = r;
    if (lane == 63) s_wcnt[wv] = ci;
    __syncthreads();

    if (wv == 0) {
      uint32_t q = lane < EW_WAVES ? s_wagg[lane] : 0u;
      uint32_t qc = lane < EW_WAVES ? s_wcnt[lane] : 0u;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t o = __shfl_up(q, 1 << d);
        uint32_t oc = __shfl_up(qc, 1 << d);
        if (lane >= (1 << d) && lane < EW_WAVES) {
          q = lds_shift(s_shift, 12 + d, o) ^ q;
          qc += oc;
        }
      }
      const uint32_t tagg = __shfl(q, EW_WAVES - 1);
      const uint32_t tcnt = __shfl(qc, EW_WAVES - 1);
      uint32_t ex = __shfl_up(q, 1);
      uint32_t exc = __shfl_up(qc, 1);
      if (lane == 0) { ex = 0; exc = 0; }
      uint32_t X;
      unsigned long long N;
      lookback(a.desc, t, tagg, tcnt, a.g_shift, X, N, a.errflag);
      if (lane < EW_WAVES) {
        uint32_t xs = X;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if ((lane >> b) & 1) xs = lds_shift(s_shift, 12 + b, xs);
        a.pwave[(uint64_t)t * EW_WAVES + lane] = xs ^ ex;
        s_wbase[lane] = N + exc;
      }
    }
    __syncthreads();
    if (cnt) write_cands(D, off, B, s_wbase[wv] + (ci - cnt), a.cpos, a.clen, a.ccap);
  }
}

// ===========================================================================
// framing: candidate links, runs, pointer jumping
// ===========================================================================
__global__ void k_link(const uint64_t *__restrict__ pos, const uint64_t *__restrict__ len, uint32_t K,
                       uint32_t *__restrict__ nxt, uint8_t *__restrict__ exc) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  const uint64_t s = pos[i] + 8 + len[i];
  uint32_t r = EW_NIL;
  if (i + 1 < K) {
    const uint64_t p1 = pos[i + 1];
    if (p1 == s) {
      r = i + 1;
    } else if (p1 < s) {
      uint32_t lo = i + 2, hi = K;
      while (lo < hi) {
        uint32_t mid = lo + ((hi - lo) >> 1);
        if (pos[mid] < s) lo = mid + 1; else hi = mid;
      }
      if (lo < K && pos[lo] == s) r = lo;
    }
  }
  nxt[i] = r;
  exc[i] = (r != i + 1);
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *E, uint32_t R, uint32_t x) {
  uint32_t lo = 0, hi = R;
  while (lo < hi) {
    uint32_t mid = lo + ((hi - lo) >> 1);
    if (E[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// run a = [E[a-1]+1, E[a]]; rs[a] = run entered after a's exit (or NIL)
__global__ void k_runs(const uint32_t *__restrict__ E, uint32_t R, const uint32_t *__restrict__ nxt,
                       uint32_t *__restrict__ rs) {
  uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= R) return;
  uint32_t n = nxt[E[a]];
  rs[a] = (n == EW_NIL) ? EW_NIL : lower_bound_u32(E, R, n);
}

__global__ void k_jump(const uint32_t *__restrict__ Jprev, uint32_t *__restrict__ Jnext, uint32_t R) {
  uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= R) return;
  uint32_t n = Jprev[a];
  Jnext[a] = (n == EW_NIL) ? EW_NIL : Jprev[n];
}

// waypoints at level k: marked a -> mark J_k(a).  Racing marks are benign:
// a node marked during this pass is an odd multiple of 2^k along the chain
// and its J_k successor is already marked.
__global__ void k_mark(const uint32_t *__restrict__ J, uint8_t *vis, uint32_t R) {
  uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= R) return;
  if (vis[a]) {
    uint32_t n = J[a];
    if (n != EW_NIL) vis[n] = 1;
  }
}

__global__ void k_entry(const uint32_t *__restrict__ E, const uint32_t *__restrict__ nxt,
                        const uint32_t *__restrict__ rs, const uint8_t *__restrict__ vis, uint32_t R,
                        uint32_t *__restrict__ entry, ChainInfo *ci) {
  uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= R) return;
  if (a == 0) entry[0] = 0;
  if (!vis[a]) return;
  uint32_t r = rs[a];
  if (r != EW_NIL) entry[r] = nxt[E[a]];
  else ci->last_cand = E[a];
}

__global__ void k_member(const uint32_t *__restrict__ E, uint32_t R, const uint8_t *__restrict__ vis,
                         const uint32_t *__restrict__ entry, uint32_t K, uint8_t *__restrict__ on) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  uint32_t a = lower_bound_u32(E, R, i);
  on[i] = (a < R && vis[a] && i >= entry[a]) ? 1 : 0;
}

// ===========================================================================
// per-frame decode (walpb.Record, raftpb.Entry, raftpb.HardState)
// ===========================================================================
__constant__ uint8_t c_kind_record[8] = {0, PB_VAR64, PB_VAR32, PB_BYTES, 0, 0, 0, 0};
__constant__ uint8_t c_kind_entry[8] = {0, PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, 0, 0, 0};
__constant__ uint8_t c_kind_state[8] = {0, PB_VAR64, PB_VAR64, PB_VAR64, 0, 0, 0, 0};

__global__ void k_decode(const uint8_t *__restrict__ buf, const uint64_t *__restrict__ pos,
                         const uint64_t *__restrict__ len, const uint32_t *__restrict__ rec_cand, uint32_t n,
                         RecDesc *__restrict__ rd) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t i = rec_cand[r];
  const uint64_t p = pos[i];
  const int64_t L = (int64_t)len[i];
  RecDesc d;
  d.off = p;
  d.type = 0; d.crc = 0; d.chained = 0; d.st = 0; d.sub_st = 0;
  d.doff = p + 8; d.dlen = 0; d.dnil = 1;
  d.f0 = d.f1 = d.f2 = 0; d.edoff = 0; d.edlen = 0; d.enil = 1; d.etype = 0;
  PbOut o;
  pb_init(o);
  int st = pb_walk(buf + p + 8, L, c_kind_record, o, nullptr, 0);
  d.type = (int64_t)o.v[1];
  d.crc = (uint32_t)o.v[2];
  if (o.blen[3] > 0) { d.doff = p + 8 + o.boff[3]; d.dlen = o.blen[3]; d.dnil = 0; }
  d.st = st;
  if (st == 0) {
    const uint8_t *dp = buf + d.doff;
    if (d.type == 2) {           // entryType: mustUnmarshalEntry
      PbOut e;
      pb_init(e);
      int s2 = d.dnil ? 0 : pb_walk(dp, (int64_t)d.dlen, c_kind_entry, e, nullptr, 0);
      if (s2 == 0 && e.unrec) s2 = 48;   // Entry.XXX_unrecognized is returned by ReadAll
      d.sub_st = s2;
      d.etype = (int32_t)(uint32_t)e.v[1];
      d.f0 = e.v[2];            // Term
      d.f1 = e.v[3];            // Index
      if (e.blen[4] > 0) { d.edoff = d.doff + e.boff[4]; d.edlen = e.blen[4]; d.enil = 0; }
    } else if (d.type == 3) {    // stateType: mustUnmarshalState
      PbOut h;
      pb_init(h);
      int s2 = d.dnil ? 0 : pb_walk(dp, (int64_t)d.dlen, c_kind_state, h, nullptr, 0);
      if (s2 == 0 && h.unrec) s2 = 48;   // HardState.XXX_unrecognized is returned
      d.sub_st = s2;
      d.f0 = h.v[1]; d.f1 = h.v[2]; d.f2 = h.v[3];
    }
  }
  rd[r] = d;
}

// Stream prefix P(x) = lin(stream[0..x)) from the per-wave prefixes and the
// per-piece lin values of k_stream.
__device__ __forceinline__ uint32_t prefix_at(uint64_t x, const uint32_t *__restrict__ pwave,
                                              const uint32_t *__restrict__ v, const uint8_t *__restrict__ buf,
                                              const uint32_t *t4, const uint32_t *s64) {
  const uint64_t w = x >> 12;
  uint32_t acc = pwave[w];
  const uint64_t x0 = x & ~(uint64_t)(EW_PIECE - 1);
  const uint32_t k = (uint32_t)((x0 >> 6) & 63);
  const uint32_t *vp = v + (w << 6);
  for (uint32_t j = 0; j < k; ++j) acc = tab_apply(s64, acc) ^ vp[j];
  return raw_bytes(t4, acc, buf, x0, x);
}

__global__ void k_verify(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pwave,
                         const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                         const uint32_t *__restrict__ g_shift, RecDesc *__restrict__ rd, uint32_t n,
                         ReadAllAgg *agg) {
  __shared__ uint32_t s_t4[1024];
  __shared__ uint32_t s_s64[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
    s_t4[i] = g_slice[i];
    s_s64[i] = g_shift[6 * 1024 + i];
  }
  __syncthreads();
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  RecDesc &d = rd[r];
  int st = d.st;
  const uint32_t seed = r ? rd[r - 1].crc : 0u;
  uint32_t chained = seed;
  if (st == 0) {
    if (d.type == 4) {                      // crcType: ReadAll's check, wal/wal.go:184-192
      if (seed != 0 && d.crc != seed) st = EWAL_ERR_WAL_CRC;
      chained = d.crc;
    } else {                                // decoder.decode: crc.Write(Data); Validate
      const uint64_t s = d.doff, e = d.doff + d.dlen;
      uint32_t computed;
      if (d.dlen == 0) {
        computed = seed;
      } else {
        const uint32_t Ps = prefix_at(s, pwave, v, buf, s_t4, s_s64);
        const uint32_t Pe = prefix_at(e, pwave, v, buf, s_t4, s_s64);
        computed = gshift_n(g_shift, d.dlen, seed ^ 0xffffffffu ^ Ps) ^ Pe ^ 0xffffffffu;
      }
      chained = computed;
      if (computed != d.crc) {
        st = EWAL_ERR_RECORD_CRC;
      } else if (d.type == 2) {
        if (d.sub_st == 48) st = EWAL_UNSUPPORTED_ENCODING;
        else if (d.sub_st == 33 || d.sub_st == 37) st = d.sub_st;
        else if (d.sub_st) st = EWAL_PANIC_ENTRY;
      } else if (d.type == 3) {
        if (d.sub_st == 48) st = EWAL_UNSUPPORTED_ENCODING;
        else if (d.sub_st == 33 || d.sub_st == 37) st = d.sub_st;
        else if (d.sub_st) st = EWAL_PANIC_STATE;
      } else if (d.type != 1) {
        st = EWAL_ERR_UNEXPECTED_TYPE;
      }
    }
  }
  d.st = st;
  d.chained = chained;
  if (st != 0) atomicMin(&agg->first_fail, (unsigned long long)r);
  if (d.type == 2) atomicMax(&agg->last_entry, (long long)r);
  if (d.type == 3) atomicMax(&agg->last_state, (long long)r);
  if (d.type == 1 && d.dlen > 0) atomicMin(&agg->first_meta, (unsigned long long)r);
}

// metadata: `metadata != nil && !reflect.DeepEqual(metadata, rec.Data)`, wal/wal.go:178-183
__global__ void k_meta(const uint8_t *__restrict__ buf, RecDesc *__restrict__ rd, uint32_t n, ReadAllAgg *agg) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const unsigned long long fm = agg->first_meta;
  if (fm == ~0ull || r <= fm) return;
  RecDesc &d = rd[r];
  if (d.type != 1 || d.st != 0) return;
  const RecDesc &m = rd[fm];
  bool eq = (d.dlen == m.dlen);
  for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = buf[d.doff + k] == buf[m.doff + k];
  if (!eq) {
    d.st = EWAL_ERR_METADATA_CONFLICT;
    atomicMin(&agg->first_fail, (unsigned long long)r);
  }
}

// entry ops: entries with Index >= ri (the `ents = append(ents[:Index-ri], e)` steps)
__global__ void k_opflag(const RecDesc *__restrict__ rd, uint32_t n, uint64_t ri, uint8_t *__restrict__ f) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const RecDesc &d = rd[r];
  f[r] = (d.type == 2 && d.st == 0 && d.f1 >= ri) ? 1 : 0;
}

// gap check: op j needs k_j <= len(ents) = k_{j-1} + 1 (wal/wal.go:173)
__global__ void k_gap(RecDesc *__restrict__ rd, const uint32_t *__restrict__ ops, uint32_t nops, uint64_t ri,
                      uint64_t *__restrict__ kk, ReadAllAgg *agg) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nops) return;
  const uint32_t r = ops[j];
  const uint64_t k = rd[r].f1 - ri;
  kk[j] = k;
  bool gap;
  if (j == 0) {
    gap = k > 0;
  } else {
    const uint64_t kp = rd[ops[j - 1]].f1 - ri;
    gap = (k > kp) && (k - kp > 1);
  }
  if (gap) {
    rd[r].st = EWAL_PANIC_INDEX_GAP;
    atomicMin(&agg->first_fail, (unsigned long long)r);
  }
}

// survivors: op j is ents[k_j] iff every later op has k > k_j
__global__ void k_ents(const RecDesc *__restrict__ rd, const uint32_t *__restrict__ ops, uint32_t nops,
                       const uint64_t *__restrict__ kk, const uint64_t *__restrict__ sufmin,
                       ewal_entry *__restrict__ ents, uint64_t nents) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nops) return;
  const uint64_t k = kk[j];
  const uint64_t later = (j + 1 < nops) ? sufmin[j + 1] : ~0ull;
  if (k < later && k < nents) {
    const RecDesc &d = rd[ops[j]];
    ewal_entry e;
    e.term = d.f0;
    e.index = d.f1;
    e.data_off = d.edoff;
    e.data_len = d.edlen;
    e.type = d.etype;
    e.data_nil = d.enil;
    ents[k] = e;
  }
}

__global__ void k_records_out(const RecDesc *__restrict__ rd, uint32_t n, ewal_record *__restrict__ out) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const RecDesc &d = rd[r];
  ewal_record o;
  o.offset = d.off;
  o.data_off = d.doff;
  o.data_len = d.dlen;
  o.type = d.type;
  o.crc = d.crc;
  o.chained_crc = d.chained;
  out[r] = o;
}

__global__ void k_reverse_u64(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint32_t n) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) out[n - 1 - j] = in[j];
}

// P(x) for one x (pkg/crc digest over a whole device buffer).
__global__ void k_prefix_one(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pwave,
                             const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                             const uint32_t *__restrict__ g_shift, uint64_t x, uint32_t *out) {
  if (threadIdx.x == 0) *out = prefix_at(x, pwave, v, buf, g_slice, g_shift + 6 * 1024);
}
