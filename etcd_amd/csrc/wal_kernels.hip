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
//   k_stream   per-lane CRC of every 64-B piece (slicing-by-4, conflict-free
//              LDS tables), lin of every 256-B super-piece -> v[], frame-start
//              candidates -> per-unit slots.
//   k_uagg / k_tscan / k_tfix / k_uapply
//              unit scan: stream prefixes P(x) = lin(stream[0..x)) at every
//              4 KiB unit, candidate bases, the dense sorted candidate list.
//   k_frame    speculative framing + decode: candidate r is frame r when the
//              candidates chain from byte 0 (checked here); canonical
//              Record / Entry / HardState parse; P at frame and data starts.
//   k_decode_slow  the general gogoprotobuf walkers for the frames k_frame
//              declined.
//   k_link, k_runs / k_jump / k_mark / k_entry / k_member, k_decode
//              the fallback framing by pointer jumping over runs of
//              consecutive candidates (false candidates, torn tails).
//   k_check    chained CRC check per frame against its predecessor's stored
//              CRC (== the reference's running CRC up to the first failure),
//              using the stream prefixes: Update(seed, D[s,e)) =
//              S_n(seed ^ ~0 ^ P(s)) ^ P(e) ^ ~0; Entry / HardState verdicts,
//              the index-gap panic, ReadAll's reductions.
//   k_result   ReadAll's metadata rule and the result gather (rare: k_gap,
//              k_ents for index gaps far back / index rewinds).
#include "ewal_device.h"
#include "ewal_internal.h"

// ===========================================================================
// k_stream
// ===========================================================================
// Slicing-by-4 tables, 32 LDS replicas, laid out so that ONE v_perm_b32 turns
// a CRC register byte into a conflict-free LDS byte address:
//   dword (t >> 1) * 16384 + b * 64 + (t & 1) * 32 + (lane & 31)
// i.e. byte address [lane byte | b << 8 | region << 16] with lane byte =
// (t & 1) * 128 + 4 * (lane & 31) and region = t >> 1.  The bank of every
// lookup is lane & 31, so a ds_read_b32 costs the minimum 2 LDS cycles.
#define EW_SLICE_DWORDS 32768   // 128 KiB
// byte k of c into address byte 1, lane byte / region from L
#define EW_PERM_SEL(k) (0x0c020000u | ((4u + (k)) << 8))
__device__ __forceinline__ uint32_t lds_lookup(const uint8_t *s, uint32_t addr) {
  return *(const uint32_t *)(s + addr);
}
__device__ __forceinline__ uint32_t slice_src(int idx) {   // g_slice index (t * 256 + b) of LDS dword idx
  const int region = idx >> 14, b = (idx >> 6) & 255, t = region * 2 + ((idx >> 5) & 1);
  return (uint32_t)(t * 256 + b);
}
// The same layout holding the byte tables of a shift S_{2^m} (table t <- byte
// 3 - t), so that the lookup step below applies S_{2^m}: g_shift index.
__device__ __forceinline__ uint32_t shift_src(int m, int idx) {
  const uint32_t tb = slice_src(idx);
  return (uint32_t)m * 1024 + (3 - (tb >> 8)) * 256 + (tb & 255);
}
// One table step on x with the data word d folded in:
//   T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3] ^ d
// (slicing tables: the CRC step; shift tables: S_{2^m}(x) ^ d).
__device__ __forceinline__ uint32_t perm_step(const uint8_t *s, const uint32_t (&Lt)[4], uint32_t x, uint32_t d) {
  const uint32_t l0 = lds_lookup(s, __builtin_amdgcn_perm(x, Lt[3], EW_PERM_SEL(0)));
  const uint32_t l1 = lds_lookup(s, __builtin_amdgcn_perm(x, Lt[2], EW_PERM_SEL(1)));
  const uint32_t l2 = lds_lookup(s, __builtin_amdgcn_perm(x, Lt[1], EW_PERM_SEL(2)));
  const uint32_t l3 = lds_lookup(s, __builtin_amdgcn_perm(x, Lt[0], EW_PERM_SEL(3)));
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(l0, l1, l2, 0x96), l3, d, 0x96);
}
__device__ __forceinline__ void lane_regs(int lane, uint32_t (&Lt)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) Lt[t] = ((uint32_t)(t >> 1) << 16) | ((uint32_t)(t & 1) << 7) | (uint32_t)((lane & 31) << 2);
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
// The per-dword pre-test is "byte p+7 == 00 (the top byte of L, 0 for every
// L <= B < 2^40) and byte p+8 == 08": a necessary condition that, unlike the
// 08 ?? 10 head alone, skips the Entry head (08 00 10) inside every entry
// record -- the byte before it ends Record.Data's length varint, never 0 --
// so record-dense streams run the exact test about half as often (configs[2]
// k_stream -9 %).
#define CAND_TEST(J)                                                                 \
  {                                                                                  \
    uint32_t x_ = D[(J) + 2];                                                        \
    uint32_t y_ = __builtin_amdgcn_alignbyte(D[(J) + 2], D[(J) + 1], 3);             \
    uint32_t z_ = (x_ ^ 0x08080808u) | y_;                                           \
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

// Branch-free filter over all 16 dword positions: nonzero iff some byte
// position may hold 08 ?? 10 at p+8 / p+10 (the exact test above then runs
// only for such lanes).  E = D ^ 08080808, so x ^ 08.. = E[J+2] and
// y ^ 10.. = alignbyte(E[J+3], E[J+2], 2) ^ 18..; one bitop3 each for z and
// for the accumulated zero-byte test.
// The pattern is CAND_TEST's pre-test, "length MSB 00 + tag 08" at p+7 / p+8:
// byte k of z = (stream byte b ^ 08) | (byte b-1), zero iff the pair
// matches.  Per dword pair: 2 alignbyte + 2 bitop3 (z) + 2 adds (the
// borrow tests) + 2 bitop3 (accumulate) = 4 VALU per dword.
__device__ __forceinline__ uint32_t cand_filter(const uint32_t (&D)[19]) {
  //   z   = (x ^ 08..) | y             bitop3 0xDE ((a ^ c) | b)
  //   acc = ((z - 01..) & ~z) | acc    bitop3 0xBA ((a & ~b) | c)
  // One accumulator per group of four dwords (J = 4g .. 4g+3), packed at
  // the end into bit 7 - g of every byte, so find_cands runs the exact test
  // only on the groups that hit (+6 VALU here, ~3/4 of the exact tests gone).
  uint32_t r = 0, acc = 0;
#pragma unroll
  for (int J = 0; J < 16; J += 2) {
    const uint32_t y0 = __builtin_amdgcn_alignbyte(D[J + 2], D[J + 1], 3);
    const uint32_t y1 = __builtin_amdgcn_alignbyte(D[J + 3], D[J + 2], 3);
    const uint32_t z0 = __builtin_amdgcn_bitop3_b32(D[J + 2], y0, 0x08080808u, 0xDE);
    const uint32_t z1 = __builtin_amdgcn_bitop3_b32(D[J + 3], y1, 0x08080808u, 0xDE);
    // z - 01.. per dword (a borrow only adds false hits, never hides a zero
    // byte; two 32-bit adds: the 64-bit form cost the compiler a register
    // pair copy and a carry add, round 5)
    const uint32_t s0 = z0 + 0xFEFEFEFFu, s1 = z1 + 0xFEFEFEFFu;
    const uint32_t a0 = __builtin_amdgcn_bitop3_b32(s0, z0, (J & 2) ? acc : 0u, 0xBA);
    acc = __builtin_amdgcn_bitop3_b32(s1, z1, a0, 0xBA);
    if (J & 2) {   // group g = J >> 2 complete: into bit 7 - g, (a & b) | c
      const int g = J >> 2;
      r = g == 0 ? (acc & 0x80808080u) : __builtin_amdgcn_bitop3_b32(acc >> g, 0x80808080u >> g, r, 0xEA);
    }
  }
  return r;
}

__device__ __forceinline__ uint32_t count_cands(const uint32_t (&D)[19], uint64_t off, uint64_t B) {
  uint32_t cnt = 0;
#define CAND_ACTION ++cnt
  CAND_TEST(0) CAND_TEST(1) CAND_TEST(2) CAND_TEST(3) CAND_TEST(4) CAND_TEST(5) CAND_TEST(6) CAND_TEST(7)
  CAND_TEST(8) CAND_TEST(9) CAND_TEST(10) CAND_TEST(11) CAND_TEST(12) CAND_TEST(13) CAND_TEST(14) CAND_TEST(15)
#undef CAND_ACTION
  return cnt;
}

// dense write of a lane's candidates (k_rescan: overflow units)
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

// slot write of a lane's candidates as 12-bit offsets inside the 4 KiB unit
__device__ __forceinline__ void slot_cands(const uint32_t (&D)[19], uint64_t off, uint64_t B, uint32_t base,
                                           uint16_t *slots, uint32_t unit_off) {
  uint32_t w = base;
#define CAND_ACTION                                                           \
  if (w < EW_SLOTS) slots[w] = (uint16_t)(unit_off + (uint32_t)(p_ - off));   \
  ++w
  CAND_TEST(0) CAND_TEST(1) CAND_TEST(2) CAND_TEST(3) CAND_TEST(4) CAND_TEST(5) CAND_TEST(6) CAND_TEST(7)
  CAND_TEST(8) CAND_TEST(9) CAND_TEST(10) CAND_TEST(11) CAND_TEST(12) CAND_TEST(13) CAND_TEST(14) CAND_TEST(15)
#undef CAND_ACTION
}

typedef uint32_t ew_v4u __attribute__((ext_vector_type(4)));
// The WAL stream is read exactly once: nontemporal loads (measured 7.0 vs
// 6.1-6.3 TB/s for the plain forms of the same read pattern, tools/membw.hip).
__device__ __forceinline__ void load_piece_fast(const uint8_t *buf, uint64_t off, uint32_t (&D)[19]) {
  const ew_v4u *p = (const ew_v4u *)(buf + off);
  ew_v4u q0 = __builtin_nontemporal_load(p), q1 = __builtin_nontemporal_load(p + 1),
         q2 = __builtin_nontemporal_load(p + 2), q3 = __builtin_nontemporal_load(p + 3);
  D[0] = q0.x; D[1] = q0.y; D[2] = q0.z; D[3] = q0.w;
  D[4] = q1.x; D[5] = q1.y; D[6] = q1.z; D[7] = q1.w;
  D[8] = q2.x; D[9] = q2.y; D[10] = q2.z; D[11] = q2.w;
  D[12] = q3.x; D[13] = q3.y; D[14] = q3.z; D[15] = q3.w;
}
// guarded form (the stream's last units, k_rescan)
__device__ __forceinline__ void load_piece(const uint8_t *buf, uint64_t B, uint64_t off, uint32_t (&D)[19]) {
  if (off + EW_PIECE <= B) {
    load_piece_fast(buf, off, D);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) D[k] = (off < B) ? load_word_guarded(buf, B, off + 4 * k) : 0u;
  }
}

// the 12 bytes after a lane's piece: the next lane's first dwords, or for
// lane 63 a direct load of the following unit
__device__ __forceinline__ void load_next3(const uint8_t *buf, uint64_t B, uint64_t off, uint32_t (&D)[19]) {
  const int lane = threadIdx.x & 63;
  D[16] = __shfl_down(D[0], 1);
  D[17] = __shfl_down(D[1], 1);
  D[18] = __shfl_down(D[2], 1);
  if (lane == 63) {
    const uint64_t o = off + EW_PIECE;
    D[16] = load_word_guarded(buf, B, o);
    D[17] = load_word_guarded(buf, B, o + 4);
    D[18] = load_word_guarded(buf, B, o + 8);
  }
}
// fast form: DPP wave_shl:1 (lane i reads lane i + 1); lane 63 keeps `old`,
// the first words of the next unit, loaded with the piece
#define EW_DPP_WAVE_SHL1 0x130
#define EW_DPP_WAVE_ROL1 0x134
typedef uint32_t ew_v3u __attribute__((ext_vector_type(3)));
__device__ __forceinline__ void next3_fast(const ew_v3u &nxt, uint32_t (&D)[19]) {
  D[16] = (uint32_t)__builtin_amdgcn_update_dpp((int)nxt.x, (int)D[0], EW_DPP_WAVE_SHL1, 0xf, 0xf, false);
  D[17] = (uint32_t)__builtin_amdgcn_update_dpp((int)nxt.y, (int)D[1], EW_DPP_WAVE_SHL1, 0xf, 0xf, false);
  D[18] = (uint32_t)__builtin_amdgcn_update_dpp((int)nxt.z, (int)D[2], EW_DPP_WAVE_SHL1, 0xf, 0xf, false);
}


// DPP controls (GFX9 family): row_shr:n = 0x110 + n, row_bcast:15 / :31.
#define EW_DPP_ROW_SHR(n) (0x110 + (n))
#define EW_DPP_ROW_BCAST15 0x142
#define EW_DPP_ROW_BCAST31 0x143
// inclusive wave prefix sum (u32), DPP only
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, EW_DPP_ROW_SHR(1), 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, EW_DPP_ROW_SHR(2), 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, EW_DPP_ROW_SHR(4), 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, EW_DPP_ROW_SHR(8), 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, EW_DPP_ROW_BCAST15, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, EW_DPP_ROW_BCAST31, 0xc, 0xf, false);
  return x;
}

// lin(piece) of NU pieces at once: slicing-by-4 chains, interleaved so the
// NU dependent chains hide each other's LDS latency.  Each step is 4 v_perm
// + 4 conflict-free ds_read_b32 + 2 v_bitop3 (the next data word folded in).
template <int NU>
__device__ __forceinline__ void crc_pieces(const uint8_t *s_slice, const uint32_t (&Lt)[4],
                                           const uint32_t (&D)[NU][19], uint32_t (&c)[NU]) {
  uint32_t x[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) x[i] = D[i][0];
#pragma unroll
  for (int k = 0; k < 16; ++k)
#pragma unroll
    for (int i = 0; i < NU; ++i) x[i] = perm_step(s_slice, Lt, x[i], k < 15 ? D[i][k + 1] : 0u);
#pragma unroll
  for (int i = 0; i < NU; ++i) c[i] = x[i];
}

// Exact test at every filter hit of a lane's piece; records the first two
// candidate offsets (12-bit, inside the unit) in registers.
__device__ __forceinline__ uint32_t find_cands(const uint32_t (&D)[19], uint32_t fm, uint64_t off, uint64_t B,
                                               uint32_t unit_off, uint32_t &pa, uint32_t &pb) {
  uint32_t n = 0;
#define CAND_ACTION                                                  \
  {                                                                  \
    const uint32_t q_ = unit_off + (uint32_t)(p_ - off);             \
    pb = (n == 1) ? q_ : pb;                                         \
    pa = (n == 0) ? q_ : pa;                                         \
    ++n;                                                             \
  }
  // only the dword groups cand_filter flagged (bit 7 - g of some byte of fm)
  if (fm & 0x80808080u) { CAND_TEST(0) CAND_TEST(1) CAND_TEST(2) CAND_TEST(3) }
  if (fm & 0x40404040u) { CAND_TEST(4) CAND_TEST(5) CAND_TEST(6) CAND_TEST(7) }
  if (fm & 0x20202020u) { CAND_TEST(8) CAND_TEST(9) CAND_TEST(10) CAND_TEST(11) }
  if (fm & 0x10101010u) { CAND_TEST(12) CAND_TEST(13) CAND_TEST(14) CAND_TEST(15) }
#undef CAND_ACTION
  return n;
}

// 4 x 4 transpose of 16-B chunks across the lane groups g = lane >> 4: on
// entry register row r (D[4r..4r+3]) of lane (g, m) holds chunk g of piece
// 16 r + m; on exit D[4c..4c+3] of lane (g, m) holds chunk c of piece
// 16 g + m, i.e. the lane owns piece `lane`.  Two butterfly stages of the
// gfx950 lane-swap instructions (v_permlane32_swap: upper half of vdst <->
// lower half of vsrc; v_permlane16_swap: odd rows of vdst <-> even rows of
// vsrc), 16 VALU per 4 KiB.
__device__ __forceinline__ void row_transpose(uint32_t (&D)[19]) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    auto s02 = __builtin_amdgcn_permlane32_swap(D[d], D[8 + d], false, false);
    auto s13 = __builtin_amdgcn_permlane32_swap(D[4 + d], D[12 + d], false, false);
    D[d] = s02[0]; D[8 + d] = s02[1];
    D[4 + d] = s13[0]; D[12 + d] = s13[1];
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    auto s01 = __builtin_amdgcn_permlane16_swap(D[d], D[4 + d], false, false);
    auto s23 = __builtin_amdgcn_permlane16_swap(D[8 + d], D[12 + d], false, false);
    D[d] = s01[0]; D[4 + d] = s01[1];
    D[8 + d] = s23[0]; D[12 + d] = s23[1];
  }
}

// EW_LOAD_HALF layout: register group r (D[4r..4r+3]) of lane (h, j) =
// (lane >> 5, lane & 31) holds chunk 2 (r >> 1) + h of piece j + 32 (r & 1).
// Swapping the upper half of group 2c with the lower half of group 2c + 1
// (one v_permlane32_swap per register) leaves chunk c of piece `lane` in
// group c, for every c.
__device__ __forceinline__ void half_transpose(uint32_t (&D)[19]) {
#pragma unroll
  for (int c = 0; c < 4; c += 2)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      auto s = __builtin_amdgcn_permlane32_swap(D[4 * c + d], D[4 * (c + 1) + d], false, false);
      D[4 * c + d] = s[0];
      D[4 * (c + 1) + d] = s[1];
    }
}

// NU units (4 KiB each, 64 B per lane) once D[i][0..18] is in registers:
// lin of every 256-B super-piece -> v[] (1/64 of the stream bytes) and
// frame-start candidates -> slots[] / wcnt[] (the unit's candidate count,
// from lane 63).  The 4 KiB aggregates are formed from v[] by k_uscan, where
// one lane per unit does it with every lane busy.
// EW_SPLIT_CAND: k_stream runs only the branch-free candidate filter and
// records which 64-B pieces it flagged (one 64-bit mask per unit); k_cand
// then runs the exact frame-start tests and writes the slots for those
// pieces alone.  In the stream pass the exact tests were divergent VALU and
// scattered slot stores on every unit of a record-dense WAL (28 % of
// k_stream on configs[2]-shaped shards, ablation EW_XS=2, r03).
#ifndef EW_SPLIT_CAND
#define EW_SPLIT_CAND 1
#endif
#ifndef EW_CAND_TAILMASK
#define EW_CAND_TAILMASK 1   // hmask also says which flagged pieces need the 16 B after them (k_cand)
#endif
#ifndef EW_LOAD_HALF
#define EW_LOAD_HALF 0   // A/B: half-used-line loads + one permlane32 stage (see k_stream)
#endif
#ifndef EW_V_NT
#define EW_V_NT 0    // A/B: v[] / hmask stored nontemporally (fewer dirty L2 lines when the stream pass ends)
#endif
// The stream pass's lin outputs (v[], vh[]) are stored with relaxed
// agent-scope atomic stores (global_store ... sc1): the lines leave the XCD's
// L2 as they are written instead of staying there dirty beside the stream's
// nontemporal loads.  Round 6 A/B, one box, the rounds before the box's
// clock state changed (profiles/r06/ab_stores_*_s4.txt): configs[1] k_stream
// 1.627 -> 1.57 ms (-3.5 %, as fast as without the v[] stores at all: the
// timing-only EW_XS=4 build, session s2), pipeline 1.957 -> 1.91 ms; 128 x 64
// MiB shards pipeline 2.922 -> 2.879 ms; configs[0] 0.2949 -> 0.2927 ms.  The
// hmask stores stay plain: as two 8-B sc1 stores by one lane (bit 4) they
// gave the gain back.  (Round 2 measured plain vs nt only.)
// (bits: 1 v[], 2 vh[], 4 hmask)
#ifndef EW_V_SC1
#define EW_V_SC1 3
#endif
template <int BIT>
__device__ __forceinline__ void st_out32(uint32_t *p, uint32_t x) {
  if (EW_V_SC1 & BIT) __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = x;
}
__device__ __forceinline__ void st_out64(unsigned long long *p, unsigned long long x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#ifndef EW_HM_PAIR
#define EW_HM_PAIR 0   // A/B: the pair loop's two hmask entries in one 2-lane store
#endif
#ifndef EW_ULIN
#define EW_ULIN 0    // A/B: k_stream stores every 4 KiB unit's lin and the frame pass's phase A loads it -- the
                     // phase A saves 18 us on configs[1], the stream pass loses 68 (+4 %, +16 % on configs[0]):
                     // off (profiles/r05/ab_notes.txt)
#endif
#ifndef EW_STREAM_AUX
#define EW_STREAM_AUX 2   // the stream pass's buffer-load cache policy: 2 = nontemporal (A/B: 0 = default policy)
#endif
#ifndef EW_RUN
#define EW_RUN 1   // A/B: consecutive pairs per wave run (1: pairs strided by the wave count)
#endif
#ifndef EW_TREE4
#define EW_TREE4 1   // the super-piece lins in one table step per lane + two DPP xors (round 5)
#endif
#ifndef EW_XS
#define EW_XS 0   // timing-only k_stream ablations (tools/): 1 no CRC, 2 no candidates, 4 no v stores,
                  // 8 the candidate filter without the exact tests / slots, 16 v stores only for
                  // units with a flagged piece; results are wrong
#endif
template <int NU, bool FIND, bool SAFE = false>   // SAFE: every piece lies inside the stream (the pair loop)
__device__ __forceinline__ void stream_units(const StreamArgs &a, const uint8_t *s_slice, const uint32_t *s_s64,
                                             const uint32_t *s_s128, const uint32_t *s_unib, const uint32_t (&Lt)[4],
                                             const uint32_t (&u)[NU], const uint32_t (&D)[NU][19]) {
  const int lane = threadIdx.x & 63;
  const uint64_t B = a.B;
  // branch-free candidate filter first: independent VALU the scheduler can
  // place in the CRC chains' LDS shadows
  uint32_t fm[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) fm[i] = (FIND && !(EW_XS & 2)) ? cand_filter(D[i]) : 0u;
  uint32_t c[NU];
  if (EW_XS & 1) {   // timing-only ablation: no CRC
#pragma unroll
    for (int i = 0; i < NU; ++i) c[i] = D[i][0] ^ D[i][5] ^ D[i][10] ^ D[i][15];
  } else {
    crc_pieces<NU>(s_slice, Lt, D, c);
  }
  const bool top = (lane & 3) == 3;
  if (FIND && a.vh) {   // record-dense WALs: every super-piece's first 128-B half, S_64(c[4m]) ^ c[4m+1] (lane 4m+1)
    const uint32_t *s64 = EW_TREE4 ? s_s64 + 2 * 1024 : s_s64;
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c[i], EW_DPP_ROW_SHR(1), 0xf, 0xf, false);
      const uint32_t h = tab_apply(s64, o) ^ c[i];
      if ((lane & 3) == 1) st_out32<2>(a.vh + (uint64_t)u[i] * EW_VPU + (lane >> 2), h);
    }
  }
#if EW_TREE4
  // lin of every 256-B super-piece (lanes 4m .. 4m+3):
  //   S_192(c[4m]) ^ S_128(c[4m+1]) ^ S_64(c[4m+2]) ^ c[4m+3]
  // lane 4m+k moves its own piece's lin by the 64 (3 - k) bytes after it --
  // ONE byte-table step through its own table (s_s64 = the four tables,
  // k = 3 the identity) -- and two DPP xors gather the quad in lane 4m+3
  // (row_shr 1 then 2: lane 4m+1 holds c'0 ^ c'1 when lane 4m+3 reads it).
  const uint32_t tb = (uint32_t)(lane & 3) * 4096u;
  const uint8_t *st = (const uint8_t *)s_s64;
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const uint32_t x = c[i];
    const uint32_t l0 = lds_lookup(st, tb | ((x << 2) & 0x3fcu));
    const uint32_t l1 = lds_lookup(st, tb | 1024u | ((x >> 6) & 0x3fcu));
    const uint32_t l2 = lds_lookup(st, tb | 2048u | ((x >> 14) & 0x3fcu));
    const uint32_t l3 = lds_lookup(st, tb | 3072u | ((x >> 22) & 0x3fcu));
    uint32_t d = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(l0, l1, l2, 0x96), l3, 0u, 0x96);
    d ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, EW_DPP_ROW_SHR(1), 0xf, 0xf, false);
    d ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, EW_DPP_ROW_SHR(2), 0xf, 0xf, false);
    c[i] = d;
  }
  (void)s_s128;
#else
  // lin of every 256-B super-piece (lanes 4m .. 4m+3) by a two-level tree,
  // branch-free: the lanes that do not combine look up entry 0 (one address,
  // a broadcast, no extra bank cycles).  Lane 4m+3 ends with the value.
  //   level 0 (odd lanes):      y = S_64(c[L-1]) ^ c[L]
  //   level 1 (lanes 3 mod 4):  z = S_128(y[L-2]) ^ y[L]
  const bool odd = lane & 1;
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c[i], EW_DPP_ROW_SHR(1), 0xf, 0xf, false);
    c[i] ^= tab_apply(s_s64, odd ? o : 0u);   // S_64(0) = 0
  }
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c[i], EW_DPP_ROW_SHR(2), 0xf, 0xf, false);
    c[i] ^= tab_apply(s_s128, top ? o : 0u);
  }
#endif
  // plain stores (measured a little faster than nontemporal ones here)
  bool vskip[NU];   // EW_XS & 16 (timing only): no v[] for units without a flagged piece
#pragma unroll
  for (int i = 0; i < NU; ++i) vskip[i] = (EW_XS & 16) && FIND && __ballot(fm[i] != 0) == 0ull;
  if (top) {
#pragma unroll
    for (int i = 0; i < NU; ++i)
      if ((!(EW_XS & 4) || c[i] == 0x12345678u) && !vskip[i]) {
        if (EW_V_NT) __builtin_nontemporal_store(c[i], a.v + (uint64_t)u[i] * EW_VPU + (lane >> 2));
        else st_out32<1>(a.v + (uint64_t)u[i] * EW_VPU + (lane >> 2), c[i]);
      }
  }
  if (FIND && EW_ULIN) {
    // the unit's lin: super-piece m's (lane 4m+3) moved by the 256 (15 - m)
    // bytes after it -- one nibble-table step through its own table -- and
    // the 16 xored into lane 63 (row_shr 4, 8 inside the rows, then the
    // row broadcasts)
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      uint32_t e = nib_apply(s_unib + (lane >> 2) * 128, top ? c[i] : 0u);
      e ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, EW_DPP_ROW_SHR(4), 0xf, 0xf, false);
      e ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, EW_DPP_ROW_SHR(8), 0xf, 0xf, false);
      e ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, EW_DPP_ROW_BCAST15, 0xa, 0xf, false);
      e ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, EW_DPP_ROW_BCAST31, 0xc, 0xf, false);
      if (lane == 63) a.ulin[u[i]] = e;
    }
  }
  if (!FIND) return;
  if (EW_SPLIT_CAND && !(EW_XS & 8)) {   // the flagged pieces, for k_cand
    if (EW_HM_PAIR && NU == 2 && SAFE && EW_CAND_TAILMASK && !EW_V_NT) {
      // the pair's two 16-B mask pairs (units u[0], u[0] + 1: 32 contiguous
      // bytes) in ONE store instruction: 1 -- lanes 0 and 1, 16 B each;
      // 2 -- lanes 0..7, one dword each (sc1 when EW_V_SC1 & 4)
      const unsigned long long hm0 = __ballot(fm[0] != 0), h30 = __ballot((fm[0] & 0x10101010u) != 0);
      const unsigned long long hm1 = __ballot(fm[NU - 1] != 0), h31 = __ballot((fm[NU - 1] & 0x10101010u) != 0);
      if (EW_HM_PAIR == 1) {
        if (lane < 2)
          *(ulonglong2 *)(a.hmask + 2 * ((uint64_t)u[0] + lane)) = lane ? make_ulonglong2(hm1, h31) : make_ulonglong2(hm0, h30);
      } else if (lane < 8) {
        const unsigned long long q = lane < 2 ? hm0 : lane < 4 ? h30 : lane < 6 ? hm1 : h31;
        st_out32<4>((uint32_t *)(a.hmask + 2 * (uint64_t)u[0]) + lane, (uint32_t)(q >> (32 * (lane & 1))));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      const uint64_t off = (uint64_t)u[i] * EW_WAVE_BYTES + (uint64_t)lane * EW_PIECE;
      const bool in = SAFE || off < B;
      const unsigned long long hm = __ballot(fm[i] != 0 && in);
      if (EW_CAND_TAILMASK) {
        // the pieces flagged in their last dword group (bit 4 of each byte
        // of fm): only their candidates can need the 12 bytes after the piece
        const unsigned long long h3 = __ballot((fm[i] & 0x10101010u) != 0 && in);
        if (lane == 0) {
          if (EW_V_NT) {
            __builtin_nontemporal_store(hm, a.hmask + 2 * (uint64_t)u[i]);
            __builtin_nontemporal_store(h3, a.hmask + 2 * (uint64_t)u[i] + 1);
          } else {
            if (EW_V_SC1 & 4) {
              st_out64(a.hmask + 2 * (uint64_t)u[i], hm);
              st_out64(a.hmask + 2 * (uint64_t)u[i] + 1, h3);
            } else {
              *(ulonglong2 *)(a.hmask + 2 * (uint64_t)u[i]) = make_ulonglong2(hm, h3);
            }
          }
        }
      } else if (lane == 0) {
        a.hmask[u[i]] = hm;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const uint64_t off = (uint64_t)u[i] * EW_WAVE_BYTES + (uint64_t)lane * EW_PIECE;
    uint32_t cnt = 0, pa = 0, pb = 0;
    if (EW_XS & 8) {   // timing-only ablation: the filter's result kept, no exact tests / slots
      if (lane == 63) a.wcnt[u[i]] = (uint32_t)__popcll(__ballot(fm[i] != 0));
      continue;
    }
    if (fm[i] && off < B) cnt = find_cands(D[i], fm[i], off, B, (uint32_t)(lane * EW_PIECE), pa, pb);
    uint32_t ci = 0;
    if (__ballot(cnt != 0)) {   // wave-uniform: most 4 KiB units hold no frame start
      ci = wave_incl_sum(cnt);
      uint16_t *sl = a.slots + (size_t)u[i] * EW_SLOTS;
      const uint32_t base = ci - cnt;
      if (cnt > 2) {
        slot_cands(D[i], off, B, base, sl, (uint32_t)(lane * EW_PIECE));
      } else {
        if (cnt >= 1 && base < EW_SLOTS) sl[base] = (uint16_t)pa;
        if (cnt >= 2 && base + 1 < EW_SLOTS) sl[base + 1] = (uint16_t)pb;
      }
    }
    if (lane == 63) a.wcnt[u[i]] = ci;
  }
}

// One HBM pass, no inter-workgroup communication.  Every wave works on PAIRS
// of adjacent units (8 KiB; pair p = units 2p, 2p + 1, grid-stride over p)
// so that two independent CRC chains hide each other's LDS latency, the
// first unit's trailing bytes come from the second unit's registers, and
// the pair's super-piece lins form one whole 128-B line of v[].  Pairs
// inside the stream (plus 16 bytes) run the unguarded loop with THREE
// register buffers: while one pair is processed the next two are in flight
// (12 waves x 16 KiB = 192 KiB of HBM reads outstanding per CU, what the HBM
// latency under full load needs).  Loop control is scalar and the loads are
// raw buffer loads (scalar base, loop-invariant lane offset), so no wait
// lands before the use.  The last units take the guarded single-unit path.
template <bool FIND>
__global__ __launch_bounds__(EW_THREADS, 1) void k_stream(StreamArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_slice[EW_SLICE_DWORDS * 4];
  __shared__ uint32_t s_unib[(FIND && EW_ULIN) ? 16 * 128 : 1];   // the unit step: S_{256 (15 - m)} nibble tables
#if EW_TREE4
  __shared__ uint32_t s_s64[4096];   // the super-piece step: S_192, S_128, S_64, identity byte tables
  uint32_t *const s_s128 = nullptr;
#else
  __shared__ uint32_t s_s64[1024], s_s128[1024];   // S_64, S_128 byte tables (super-piece tree)
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  static_assert(sizeof(Small) % 4 == 0 && sizeof(Small) / 4 <= EW_THREADS, "Small is zeroed by one workgroup");
  if (blockIdx.x == 0 && a.u_begin == 0 && tid < (int)(sizeof(Small) / 4)) ((uint32_t *)a.small)[tid] = 0u;   // the call's scratch
  uint32_t Lt[4];
  lane_regs(lane, Lt);
  const uint64_t B = a.B;
  const uint32_t W = gridDim.x * EW_WAVES;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t p0 = blockIdx.x * EW_WAVES + wv;
  const uint32_t nsafe = B >= 16 ? (uint32_t)std::min<uint64_t>(a.nunits, (B - 16) / EW_WAVE_BYTES) : 0u;
  // pairs whose units are both safe, inside this launch's units [u_begin, u_end)
  const uint32_t PB = a.u_begin / 2;
  const uint32_t NP = std::max(PB, std::min(nsafe / 2, a.u_end / 2));
  // Unit loads are fully coalesced: load r covers unit bytes [1024 r, 1024 r + 1024)
  // with lane (g, m) = (lane >> 4, lane & 15) taking chunk g of piece 16 r + m
  // (a permutation inside the 1 KiB row, measured as fast as the plain order).
  // row_transpose() then gives every lane the 64 contiguous bytes of piece `lane`.
#if EW_LOAD_HALF
  // A/B variant: lane (h, j) = (lane >> 5, lane & 31) loads chunk c + h of
  // piece j (and of piece 32 + j, 2 KiB on) -- 16 half-used lines per load
  // instead of 8 whole ones -- so ONE permlane32 stage puts piece `lane` in
  // every lane (half_transpose: 8 swaps per unit instead of 16)
  const uint32_t lo = (uint32_t)(64 * (lane & 31) + 16 * (lane >> 5));
#else
  const uint32_t lo = (uint32_t)(64 * (lane & 15) + 16 * (lane >> 4));
#endif
  // Raw buffer loads: the pair base lives in the (scalar) buffer resource,
  // the per-lane offset is a loop-invariant VGPR, so no address VGPR is ever
  // rewritten while loads are in flight.  Lane 63 also fetches the 12 bytes
  // after the pair; the other lanes' offset for that load is out of range
  // (the resource covers 8192 + 12 bytes), which returns 0 and moves no data.
  const int o3 = lane == 63 ? 2 * EW_WAVE_BYTES : 0x7ffffff0;
  auto load_pair = [&](uint32_t p, uint32_t (&T)[2][19], ew_v3u &t3) {
    p = __builtin_amdgcn_readfirstlane(p);
    const uint8_t *pb = a.buf + (uint64_t)p * (2 * EW_WAVE_BYTES);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)pb, 0, 2 * EW_WAVE_BYTES + 12, 0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#if EW_LOAD_HALF   // register group r: chunk c = 2 (r >> 1) (+ h) of piece j + 32 (r & 1)
        const int off = EW_WAVE_BYTES * i + 2048 * (r & 1) + 32 * (r >> 1);
#else
        const int off = EW_WAVE_BYTES * i + 1024 * r;
#endif
        const ew_v4u w = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)lo + off, 0, EW_STREAM_AUX);
        T[i][4 * r] = w.x; T[i][4 * r + 1] = w.y; T[i][4 * r + 2] = w.z; T[i][4 * r + 3] = w.w;
      }
    }
    t3 = __builtin_amdgcn_raw_buffer_load_b96(rs, o3, 0, EW_STREAM_AUX);
  };
  auto run_pair = [&](uint32_t p, uint32_t (&T)[2][19], const ew_v3u &t3) {
#if EW_LOAD_HALF
    half_transpose(T[0]);
    half_transpose(T[1]);
#else
    row_transpose(T[0]);
    row_transpose(T[1]);
#endif
    // unit 0's lane 63 continues into unit 1's piece 0 (lane 0): wave_rol:1
    ew_v3u f3;
    f3.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)T[1][0], EW_DPP_WAVE_ROL1, 0xf, 0xf, false);
    f3.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)T[1][1], EW_DPP_WAVE_ROL1, 0xf, 0xf, false);
    f3.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)T[1][2], EW_DPP_WAVE_ROL1, 0xf, 0xf, false);
    next3_fast(f3, T[0]);
    next3_fast(t3, T[1]);
    const uint32_t uu[2] = {2 * p, 2 * p + 1};
    stream_units<2, FIND, true>(a, s_slice, s_s64, s_s128, s_unib, Lt, uu, T);
  };
#if EW_RUN > 1
  // A/B (EW_RUN = R): each wave takes runs of R consecutive pairs, the runs
  // dealt round-robin over the waves (span W * R pairs), instead of single
  // pairs strided by W
  const uint32_t tot = NP > PB ? NP - PB : 0u, span = W * EW_RUN;
  const uint32_t remr = tot % span, myr = p0 * EW_RUN;
  const uint32_t npairs = (tot / span) * EW_RUN + (remr > myr ? std::min<uint32_t>(remr - myr, EW_RUN) : 0u);
  auto pair_at = [&](uint32_t k) {
    const uint32_t kk = k < npairs ? k : npairs - 1;
    return __builtin_amdgcn_readfirstlane(PB + (kk / EW_RUN) * span + myr + kk % EW_RUN);
  };
#else
  const uint32_t npairs = PB + p0 < NP ? (NP - 1 - PB - p0) / W + 1 : 0u;
  auto pair_at = [&](uint32_t k) {   // clamped: a prefetch past the end reloads the last pair
    return __builtin_amdgcn_readfirstlane(PB + p0 + W * (k < npairs ? k : npairs - 1));
  };
#endif
  uint32_t DA[2][19], DB[2][19], DC[2][19];
  ew_v3u nA, nB, nC;
  if (npairs) {   // the first two pairs are in flight while the tables are staged
    load_pair(pair_at(0), DA, nA);
    load_pair(pair_at(1), DB, nB);
  }
  stage_lds<EW_THREADS>((uint32_t *)s_slice, EW_SLICE_DWORDS, [&](int i) { return a.g_slice[slice_src(i)]; });
  if (FIND && EW_ULIN) stage_lds<EW_THREADS>(s_unib, 16 * 128, [&](int i) { return a.g_unib[i]; });
#if EW_TREE4
  stage_lds<EW_THREADS>(s_s64, 4096, [&](int i) {
    const int k = i >> 10, j = i & 1023;   // table k of lane class k; j = t * 256 + b: S(b << 8t)
    if (k == 3) return (uint32_t)(j & 255) << (8 * (j >> 8));
    if (k == 2) return a.g_shift[6 * 1024 + j];
    if (k == 1) return a.g_shift[7 * 1024 + j];
    return tab_apply(a.g_shift + 7 * 1024, a.g_shift[6 * 1024 + j]);   // S_192 = S_128 . S_64
  });
#else
  stage_lds<EW_THREADS>(s_s64, 1024, [&](int i) { return a.g_shift[6 * 1024 + i]; });
  stage_lds<EW_THREADS>(s_s128, 1024, [&](int i) { return a.g_shift[7 * 1024 + i]; });
#endif
  __syncthreads();
  // sched_barrier: each batch of loads stays ahead of the previous pair's arithmetic
  for (uint32_t k = 0; k < npairs; k += 3) {   // A is processed while B and C load, and so on
    load_pair(pair_at(k + 2), DC, nC);
    __builtin_amdgcn_sched_barrier(0);
    run_pair(pair_at(k), DA, nA);
    if (k + 1 >= npairs) break;
    load_pair(pair_at(k + 3), DA, nA);
    __builtin_amdgcn_sched_barrier(0);
    run_pair(pair_at(k + 1), DB, nB);
    if (k + 2 >= npairs) break;
    load_pair(pair_at(k + 4), DB, nB);
    __builtin_amdgcn_sched_barrier(0);
    run_pair(pair_at(k + 2), DC, nC);
  }
  for (uint32_t u = std::max(2 * NP, a.u_begin) + p0; u < a.u_end; u += W) {
    const uint64_t off = (uint64_t)u * EW_WAVE_BYTES + (uint64_t)lane * EW_PIECE;
    uint32_t D1[1][19];
    load_piece(a.buf, B, off, D1[0]);
    load_next3(a.buf, B, off, D1[0]);
    const uint32_t uu[1] = {u};
    stream_units<1, FIND>(a, s_slice, s_s64, s_s128, s_unib, Lt, uu, D1);
  }
}

// ===========================================================================
// k_cand (EW_SPLIT_CAND): the exact frame-start test on the 64-B pieces
// k_stream's filter flagged, and every unit's slots and candidate count.
// One wave per 64 G units: lane l reads unit l's masks, the wave lists the
// flagged pieces (unit, piece) in order in LDS, then takes them 64 at a
// time -- each lane loads its piece plus the 12 bytes after it (80 B), runs
// the filter and the exact tests, and places its candidates after those of
// the unit's earlier pieces (a segmented scan over the round, the unit's
// running count in LDS), so every unit's slots stay position-sorted.
// ===========================================================================
#define EW_CAND_WAVES 4
#define EW_CAND_PF 4      // rounds of 64 flagged pieces whose loads are in flight together
// the piece alone (its last dword group held no flag: every candidate's head
// bytes lie inside it); the 12 bytes after it read as zeros, which no filter
// or exact test matches
__device__ __forceinline__ void load_piece64(const uint8_t *buf, uint64_t B, uint64_t off, uint32_t (&D)[19]) {
  if (off + 64 <= B) {
    const uint4 *q = (const uint4 *)(buf + off);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 x = q[k];
      D[4 * k] = x.x; D[4 * k + 1] = x.y; D[4 * k + 2] = x.z; D[4 * k + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) D[k] = load_word_guarded(buf, B, off + 4 * k);
  }
  D[16] = D[17] = D[18] = 0u;
}
__device__ __forceinline__ void load_piece80(const uint8_t *buf, uint64_t B, uint64_t off, uint32_t (&D)[19]) {
  if (off + 80 <= B) {
    const uint4 *q = (const uint4 *)(buf + off);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 x = q[k];
      D[4 * k] = x.x; D[4 * k + 1] = x.y; D[4 * k + 2] = x.z; D[4 * k + 3] = x.w;
    }
    const uint4 x = q[4];
    D[16] = x.x; D[17] = x.y; D[18] = x.z;
  } else {
#pragma unroll
    for (int k = 0; k < 19; ++k) D[k] = load_word_guarded(buf, B, off + 4 * k);
  }
}
// G groups of 64 units per wave (G = 4 when the stream has enough units to
// fill the GPU that way): the flagged pieces of consecutive groups share one
// list of up to 4096 entries, so a sparse WAL's wave issues the piece loads of
// 256 units in one round trip instead of four.
template <int G>
__global__ __launch_bounds__(EW_CAND_WAVES * 64) void k_cand(const uint8_t *__restrict__ buf, uint64_t B,
                                                             uint32_t nunits,
                                                             const unsigned long long *__restrict__ hmask,
                                                             uint16_t *__restrict__ slots,
                                                             uint32_t *__restrict__ wcnt) {
  __shared__ uint16_t s_list[EW_CAND_WAVES][64 * 64];
  __shared__ uint32_t s_ucnt[EW_CAND_WAVES][64 * G];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u0 = (blockIdx.x * EW_CAND_WAVES + (uint32_t)wv) * 64 * G;   // the wave's first unit
  uint16_t *list = s_list[wv];
  uint32_t *ucnt = s_ucnt[wv];
  unsigned long long hm[G], h3[G];   // flagged pieces; those of them that need the 16 B after the piece
  uint32_t pc[G], ex[G], Tg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t ul = u0 + 64 * g + (uint32_t)lane;
    if (EW_CAND_TAILMASK) {
      const ulonglong2 hh = ul < nunits ? *(const ulonglong2 *)(hmask + 2 * (uint64_t)ul) : make_ulonglong2(0ull, 0ull);
      hm[g] = hh.x;
      h3[g] = hh.y;
    } else {
      hm[g] = ul < nunits ? hmask[ul] : 0ull;
      h3[g] = hm[g];
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    pc[g] = (uint32_t)__popcll(hm[g]);
    const uint32_t incl = wave_incl_sum(pc[g]);
    ex[g] = incl - pc[g];
    Tg[g] = (uint32_t)__shfl((int)incl, 63);
    ucnt[64 * g + lane] = 0;
  }
  // chunks of consecutive groups whose flagged pieces fit the list (a group
  // alone always does: 64 units x 64 pieces); Tg are wave-uniform
  uint32_t gb = 0;
  while (gb < (uint32_t)G) {
    uint32_t T = 0, ge = gb;
#pragma unroll
    for (int g = 0; g < G; ++g)
      if ((uint32_t)g == ge && ge < (uint32_t)G && T + Tg[g] <= 64 * 64) { T += Tg[g]; ++ge; }
    if (T) {
      uint32_t base = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if ((uint32_t)g < gb || (uint32_t)g >= ge) continue;
        uint32_t k = base + ex[g];
        unsigned long long m = hm[g];
        while (m) {
          const int b = __ffsll((long long)m) - 1;
          m &= m - 1;
          // (unit in the wave, piece, bit 15: the 16 B after it are needed)
          list[k++] = (uint16_t)(((64 * g + lane) << 6) | b | (((h3[g] >> b) & 1ull) << 15));
        }
        base += Tg[g];
      }
      // the list and the counts are this wave's alone: a wave-level fence
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // up to EW_CAND_PF rounds of pieces in flight at once, then processed in order
      for (uint32_t rb = 0; rb < T; rb += 64 * EW_CAND_PF) {
        uint32_t D[EW_CAND_PF][19], E[EW_CAND_PF];
#pragma unroll
        for (int k = 0; k < EW_CAND_PF; ++k) {
          const uint32_t i = rb + 64 * k + (uint32_t)lane;
          E[k] = i < T ? list[i] : 0xffffu;
          if (i < T) {
            const uint64_t po = (uint64_t)(u0 + ((E[k] & 0x7fffu) >> 6)) * EW_WAVE_BYTES + (uint64_t)(E[k] & 63) * EW_PIECE;
            if (E[k] & 0x8000u) load_piece80(buf, B, po, D[k]);
            else load_piece64(buf, B, po, D[k]);   // no candidate can reach past the piece
            E[k] &= 0x7fffu;
          } else {
#pragma unroll
            for (int q = 0; q < 19; ++q) D[k][q] = 0u;
          }
        }
#pragma unroll
        for (int k = 0; k < EW_CAND_PF; ++k) {
          const uint32_t r0 = rb + 64 * k;
          if (r0 >= T) break;   // wave-uniform
          const uint32_t i = r0 + (uint32_t)lane;
          const bool live = i < T;
          const uint32_t e = E[k];
          const uint32_t ulo = e >> 6, pcs = e & 63;
          const uint64_t off = (uint64_t)(u0 + ulo) * EW_WAVE_BYTES + (uint64_t)pcs * EW_PIECE;
          uint32_t pa = 0, pb = 0, cnt = 0;
          if (live) {
            const uint32_t fm = cand_filter(D[k]);
            if (fm) cnt = find_cands(D[k], fm, off, B, pcs * EW_PIECE, pa, pb);
          }
          // segmented exclusive scan of cnt over the round (a unit's pieces are contiguous)
          const uint32_t incl = wave_incl_sum(cnt);
          const uint32_t prev = (uint32_t)__shfl_up((int)e, 1);
          const bool head = lane == 0 || (prev >> 6) != ulo;
          const unsigned long long H = __ballot(head);
          const int hl = 63 - __clzll((long long)(H & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull))));
          const uint32_t before = (uint32_t)__shfl((int)incl, hl > 0 ? hl - 1 : 0);
          const uint32_t sbase = (live ? ucnt[ulo] : 0u) + (incl - cnt - (hl > 0 ? before : 0u));
          const uint32_t nxt = (uint32_t)__shfl_down((int)e, 1);
          const bool last = live && (lane == 63 || i + 1 >= T || (nxt >> 6) != ulo);
          if (last) ucnt[ulo] = sbase + cnt;
          if (cnt) {
            uint16_t *sl = slots + (size_t)(u0 + ulo) * EW_SLOTS;
            if (cnt > 2) {
              slot_cands(D[k], off, B, sbase, sl, pcs * EW_PIECE);
            } else {
              if (sbase < EW_SLOTS) sl[sbase] = (uint16_t)pa;
              if (cnt >= 2 && sbase + 1 < EW_SLOTS) sl[sbase + 1] = (uint16_t)pb;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
    gb = ge > gb ? ge : gb + 1;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t ul = u0 + 64 * g + (uint32_t)lane;
    if (ul < nunits) wcnt[ul] = ucnt[64 * g + lane];
  }
}

// ===========================================================================
// unit scan: stream prefixes P at every 4 KiB unit, candidate bases, and the
// dense candidate list -- three launches, no inter-workgroup waiting:
//   k_uagg   per 4 MiB tile (1024 units, one workgroup): each unit's
//            aggregate lin(4 KiB) from its 16 super-piece lins v[] (Horner
//            with S_256 joined with S_1024) -> ux[u]; the tile's affine
//            aggregate and candidate count -> tagg[t], tcnt[t]
//   k_tscan  one workgroup scans the tile aggregates -> tpx[t] (P at the
//            tile start), tcb[t] (candidates before the tile), *total
//   k_uapply per tile: the in-tile scan of ux / wcnt on top of the tile's
//            prefix -> pwave[u], cbase[u]; compacts the unit's candidate
//            slots into cpos[] (units with more than EW_SLOTS: k_rescan)
// ===========================================================================

// The unit scan turns the per-unit lins into the stream prefix P at every
// unit start.  Three kernels, one WAVE per 1 MiB tile (EW_TILE_UNITS = 256
// units) so no workgroup barrier sits on the critical path:
//   k_uagg   per-unit lin x (from the 16 super-piece lins) and per-tile
//            aggregate, via the linear form  agg = XOR_u S_{4096 (255-u)}(x_u);
//   k_tscan  exclusive affine scan of the tile aggregates (one workgroup);
//   k_uapply lane-serial Horner over 4 consecutive units, one wave scan of
//            the 64 lane spans, replay -> P and candidate base per unit, and
//            the candidate-list compaction.
#define EW_TILE_UNITS 256
#define EW_TILE_LOG 20                            // 1 MiB

// Lane l of a wave reads units 64 i + l (i = 0..3: coalesced 4 KiB rows of
// v), forms x with 15 S_256 steps through the conflict-free perm-layout table
// (the k_stream layout: 128 KiB, bank = lane & 31), folds its 4 units with
// h = S_{2^18}(h) ^ x (S_{2^18} = 64 units), shifts the fold by the units
// after it in its row (S_{4096 (63-l)}) and XOR-reduces.  One workgroup of
// 16 waves per CU, persistent over the tiles.
__global__ __launch_bounds__(1024, 1) void k_uagg(ScanArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_s256[EW_SLICE_DWORDS * 4];   // S_256, perm layout
  __shared__ uint32_t s_sh[7 * 1024];             // S_{2^12} .. S_{2^18}
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint4 q[4][4];
  uint32_t c[4];
  auto load_tile = [&](uint32_t t) {   // every load of the tile up front
    const uint32_t u0 = t * EW_TILE_UNITS + lane;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t u = u0 + 64 * r;
      const bool in = u < a.nunits;
      const uint4 *vq = (const uint4 *)(a.v + (size_t)(in ? u : 0) * EW_VPU);
#pragma unroll
      for (int g = 0; g < 4; ++g) q[r][g] = in ? vq[g] : make_uint4(0, 0, 0, 0);
      c[r] = in ? a.wcnt[u] : 0u;
    }
  };
  const uint32_t t0 = blockIdx.x * 16 + wv, tstride = gridDim.x * 16;
  if (t0 < a.ntiles) load_tile(t0);   // in flight while the tables are staged
  stage_lds<1024>((uint32_t *)s_s256, EW_SLICE_DWORDS, [&](int i) { return a.g_shift[shift_src(EW_VLOG, i)]; });
  stage_lds<1024>(s_sh, 7 * 1024, [&](int i) { return a.g_shift[12 * 1024 + i]; });
  __syncthreads();
  uint32_t Lt[4];
  lane_regs(lane, Lt);
  for (uint32_t t = t0; t < a.ntiles; t += tstride) {
    const uint32_t u0 = t * EW_TILE_UNITS + lane;
    if (t != t0) load_tile(t);
    uint32_t x[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = q[r][0].x;
#pragma unroll
    for (int k = 1; k < 16; ++k)   // four independent Horner chains
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint4 &g = q[r][k >> 2];
        const uint32_t d = (k & 3) == 0 ? g.x : (k & 3) == 1 ? g.y : (k & 3) == 2 ? g.z : g.w;
        x[r] = perm_step(s_s256, Lt, x[r], d);
      }
    uint32_t h = 0, cnt = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (u0 + 64 * r < a.nunits) a.ux[u0 + 64 * r] = x[r];
      h = tab_apply(s_sh + 6 * 1024, h) ^ x[r];
      cnt += c[r];
    }
    const uint32_t after = 63 - lane;
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if ((after >> k) & 1) h = tab_apply(s_sh + k * 1024, h);
#pragma unroll
    for (int o = 32; o; o >>= 1) {
      h ^= __shfl_xor(h, o);
      cnt += __shfl_xor(cnt, o);
    }
    if (lane == 0) { a.tagg[t] = h; a.tcnt[t] = cnt; }
  }
}

// Tile scan in two launches of one workgroup per 1024 tiles (1 GiB):
//   k_tscan  thread T <- tile 1024 b + T: wave and workgroup scans of the tile
//            aggregates (S_{2^(20+d)}), the exclusive in-group prefix -> tpx,
//            tcb, the group aggregate -> gagg[b], gcnt[b];
//   k_tfix   P at the group start from the groups before it, via the linear
//            form XOR_i S_{2^30 (b-1-i)}(gagg[i]) (thread i, workgroup XOR), then
//            tpx[t] = S_{2^20 T}(P at the group start) ^ tpx[t].
__global__ __launch_bounds__(1024) void k_tscan(ScanArgs a) {
  __shared__ uint32_t s_sh[10 * 1024];            // S_{2^20} .. S_{2^29}
  __shared__ uint32_t s_wq[16];
  __shared__ unsigned long long s_wc[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  stage_lds<1024>(s_sh, 10 * 1024, [&](int i) { return a.g_shift[EW_TILE_LOG * 1024 + i]; });
  __syncthreads();
  const uint32_t t = blockIdx.x * 1024 + tid;
  const bool in = t < a.ntiles;
  uint32_t q = in ? a.tagg[t] : 0u;
  unsigned long long qc = in ? a.tcnt[t] : 0u;
#pragma unroll
  for (int d = 0; d < 6; ++d) {
    const uint32_t o = __shfl_up(q, 1 << d);
    const unsigned long long oc = __shfl_up(qc, 1 << d);
    if (lane >= (1 << d)) { q = tab_apply(s_sh + d * 1024, o) ^ q; qc += oc; }
  }
  uint32_t ex = __shfl_up(q, 1);
  unsigned long long exc = __shfl_up(qc, 1);
  if (lane == 0) { ex = 0; exc = 0; }
  if (lane == 63) { s_wq[wv] = q; s_wc[wv] = qc; }
  __syncthreads();
  if (wv == 0) {   // scan of the 16 wave spans, in place (exclusive)
    uint32_t w = lane < 16 ? s_wq[lane] : 0u;
    unsigned long long wc = lane < 16 ? s_wc[lane] : 0ull;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t o = __shfl_up(w, 1 << d);
      const unsigned long long oc = __shfl_up(wc, 1 << d);
      if (lane >= (1 << d) && lane < 16) { w = tab_apply(s_sh + (6 + d) * 1024, o) ^ w; wc += oc; }
    }
    uint32_t we = __shfl_up(w, 1);
    unsigned long long wce = __shfl_up(wc, 1);
    if (lane == 0) { we = 0; wce = 0; }
    if (lane == 15) { a.gagg[blockIdx.x] = w; a.gcnt[blockIdx.x] = wc; }
    if (lane < 16) { s_wq[lane] = we; s_wc[lane] = wce; }
  }
  __syncthreads();
  uint32_t cur = s_wq[wv];                        // S_{2^20 lane}(wave start) ^ lane prefix
#pragma unroll
  for (int b = 0; b < 6; ++b)
    if ((lane >> b) & 1) cur = tab_apply(s_sh + b * 1024, cur);
  if (in) {
    a.tpx[t] = cur ^ ex;
    a.tcb[t] = s_wc[wv] + exc;
  }
}

__global__ __launch_bounds__(1024) void k_tfix(ScanArgs a, uint32_t ngroups) {
  __shared__ uint32_t s_sh[20 * 1024];            // S_{2^20} .. S_{2^39}
  __shared__ uint32_t s_x[16];
  __shared__ unsigned long long s_c[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t b = blockIdx.x;
  if (b == 0 && ngroups == 1) {
    if (tid == 0) *a.total = a.gcnt[0];
    return;                                       // one group: tpx is final
  }
  stage_lds<1024>(s_sh, 20 * 1024, [&](int i) { return a.g_shift[EW_TILE_LOG * 1024 + i]; });
  __syncthreads();
  // group i < b contributes S_{2^30 (b - 1 - i)}(gagg[i]); groups <= 1024
  uint32_t x = 0;
  unsigned long long cnt = 0;
  if ((uint32_t)tid < b) {
    x = a.gagg[tid];
    cnt = a.gcnt[tid];
    const uint32_t m = b - 1 - tid;
#pragma unroll
    for (int k = 0; k < 10; ++k)
      if ((m >> k) & 1) x = tab_apply(s_sh + (10 + k) * 1024, x);
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    x ^= __shfl_xor(x, o);
    cnt += __shfl_xor(cnt, o);
  }
  if (lane == 0) { s_x[wv] = x; s_c[wv] = cnt; }
  __syncthreads();
  uint32_t P = 0;
  unsigned long long C = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) { P ^= s_x[w]; C += s_c[w]; }
  if (b == ngroups - 1 && tid == 0) *a.total = C + a.gcnt[b];
  if (b == 0) return;                             // P = 0 at the stream start
  const uint32_t t = b * 1024 + tid;
  if (t < a.ntiles) {
#pragma unroll
    for (int k = 0; k < 10; ++k)
      if ((tid >> k) & 1) P = tab_apply(s_sh + k * 1024, P);
    a.tpx[t] ^= P;
    a.tcb[t] += C;
  }
}

// Lane l owns units 4 l .. 4 l + 3 of the wave's tile: Horner over them
// (S_4096), wave scan of the 64 lane spans (S_{2^(14+d)}), lane start =
// S_{2^14 l}(P at the tile start) ^ exclusive span, replay.
// One persistent 16-wave workgroup per CU (each stages the 28 KiB of tables
// once; four-wave workgroups, one per tile group, staged them 2048 times for
// configs[1]).
__global__ __launch_bounds__(1024) void k_uapply(ScanArgs a) {
  __shared__ uint32_t s_s12[1024];                // S_4096
  __shared__ uint32_t s_sh[6 * 1024];             // S_{2^14} .. S_{2^19}
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  stage_lds<1024>(s_s12, 1024, [&](int i) { return a.g_shift[12 * 1024 + i]; });
  stage_lds<1024>(s_sh, 6 * 1024, [&](int i) { return a.g_shift[14 * 1024 + i]; });
  __syncthreads();
  for (uint32_t t = blockIdx.x * 16 + wv; t < a.ntiles; t += gridDim.x * 16) {
    const uint32_t u0 = t * EW_TILE_UNITS + 4 * lane;
    const bool full = u0 + 4 <= a.nunits;
    uint32_t x[4], c[4];
    if (full) {
      const uint4 xv = *(const uint4 *)(a.ux + u0), cv = *(const uint4 *)(a.wcnt + u0);
      x[0] = xv.x; x[1] = xv.y; x[2] = xv.z; x[3] = xv.w;
      c[0] = cv.x; c[1] = cv.y; c[2] = cv.z; c[3] = cv.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool in = u0 + j < a.nunits;
        x[j] = in ? a.ux[u0 + j] : 0u;
        c[j] = in ? a.wcnt[u0 + j] : 0u;
      }
    }
    // the tile's P / base and the first 8 candidate slots of every unit with
    // candidates, issued before the arithmetic so the wave waits once
    const uint32_t tp = a.tpx[t];
    const unsigned long long tcb = a.tcb[t];
    uint4 sv[4];
    if (a.slots) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        sv[j] = c[j] ? *(const uint4 *)(a.slots + (size_t)(u0 + j) * EW_SLOTS) : make_uint4(0, 0, 0, 0);
    }
    uint32_t q = 0, qc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) { q = tab_apply(s_s12, q) ^ x[j]; qc += c[j]; }
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      const uint32_t o = __shfl_up(q, 1 << d), oc = __shfl_up(qc, 1 << d);
      if (lane >= (1 << d)) { q = tab_apply(s_sh + d * 1024, o) ^ q; qc += oc; }
    }
    uint32_t ex = __shfl_up(q, 1), exc = __shfl_up(qc, 1);
    if (lane == 0) { ex = 0; exc = 0; }
    uint32_t cur = tp;
#pragma unroll
    for (int b = 0; b < 6; ++b)
      if ((lane >> b) & 1) cur = tab_apply(s_sh + b * 1024, cur);
    cur ^= ex;
    unsigned long long cb = tcb + exc;
    uint32_t pw[4];
    unsigned long long cbs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pw[j] = cur;
      cbs[j] = cb;
      cur = tab_apply(s_s12, cur) ^ x[j];
      cb += c[j];
    }
    if (full) {
      *(uint4 *)(a.pwave + u0) = make_uint4(pw[0], pw[1], pw[2], pw[3]);
      ulonglong2 w0, w1;
      w0.x = cbs[0]; w0.y = cbs[1]; w1.x = cbs[2]; w1.y = cbs[3];
      ((ulonglong2 *)(a.cbase + u0))[0] = w0;
      ((ulonglong2 *)(a.cbase + u0))[1] = w1;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (u0 + j < a.nunits) { a.pwave[u0 + j] = pw[j]; a.cbase[u0 + j] = cbs[j]; }
    }
    if (a.slots) {   // compaction: slots -> the dense, position-sorted candidate list
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t u = u0 + j, cx = c[j];
        if (!cx) continue;
        if (cx > EW_SLOTS) {
          a.ovf[atomicAdd(a.novf, 1u)] = u;
        } else {
          const uint64_t ub = (uint64_t)u * EW_WAVE_BYTES;
          const uint32_t w4[4] = {sv[j].x, sv[j].y, sv[j].z, sv[j].w};
#pragma unroll
          for (uint32_t m = 0; m < 8; ++m)
            if (m < cx && cbs[j] + m < a.ccap) a.cpos[cbs[j] + m] = ub + ((w4[m >> 1] >> (16 * (m & 1))) & 0xffffu);
          if (cx > 8) {   // more than 8 candidates in 4 KiB (small records): the rest of the
                          // slot line in three loads up front (a load / store loop here waits on
                          // every load in turn: cpos may alias slots)
            const uint4 *sq = (const uint4 *)(a.slots + (size_t)u * EW_SLOTS);
            const uint4 t1 = sq[1], t2 = sq[2], t3 = sq[3];
            const uint32_t w24[12] = {t1.x, t1.y, t1.z, t1.w, t2.x, t2.y, t2.z, t2.w, t3.x, t3.y, t3.z, t3.w};
#pragma unroll
            for (uint32_t m = 8; m < EW_SLOTS; ++m)
              if (m < cx && cbs[j] + m < a.ccap)
                a.cpos[cbs[j] + m] = ub + ((w24[(m - 8) >> 1] >> (16 * (m & 1))) & 0xffffu);
          }
        }
      }
    }
  }
}

__device__ __forceinline__ uint64_t ld_le64(const uint8_t *p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// slots -> the dense, position-sorted candidate list
__global__ void k_compact(const uint8_t *__restrict__ buf, uint32_t nunits, const uint32_t *__restrict__ wcnt,
                          const unsigned long long *__restrict__ cbase, const uint16_t *__restrict__ slots,
                          uint64_t *__restrict__ cpos, uint64_t *__restrict__ clen, uint64_t ccap,
                          uint32_t *__restrict__ ovf, uint32_t *novf) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits) return;
  const uint32_t cnt = wcnt[u];
  if (cnt == 0) return;
  if (cnt > EW_SLOTS) {
    ovf[atomicAdd(novf, 1u)] = u;
    return;
  }
  const unsigned long long base = cbase[u];
  for (uint32_t j = 0; j < cnt; ++j) {
    const uint64_t p = (uint64_t)u * EW_WAVE_BYTES + slots[(size_t)u * EW_SLOTS + j];
    if (base + j < ccap) {
      cpos[base + j] = p;
      clen[base + j] = ld_le64(buf + p);
    }
  }
}

// units with more than EW_SLOTS candidates: one wave re-derives them
__global__ void k_rescan(const uint8_t *__restrict__ buf, uint64_t B, const uint32_t *__restrict__ ovf,
                         const uint32_t *novf, const unsigned long long *__restrict__ cbase,
                         uint64_t *__restrict__ cpos, uint64_t *__restrict__ clen, uint64_t ccap) {
  const int lane = threadIdx.x & 63;
  const uint32_t n = *novf;
  const uint32_t W = gridDim.x * (blockDim.x >> 6);
  for (uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += W) {
    const uint32_t u = ovf[i];
    const uint64_t off = (uint64_t)u * EW_WAVE_BYTES + (uint64_t)lane * EW_PIECE;
    uint32_t D[19];
    load_piece(buf, B, off, D);
    load_next3(buf, B, off, D);
    const uint32_t cnt = off < B ? count_cands(D, off, B) : 0u;
    uint32_t ci = cnt;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      uint32_t o = __shfl_up(ci, 1 << d);
      if (lane >= (1 << d)) ci += o;
    }
    if (cnt) write_cands(D, off, B, cbase[u] + (ci - cnt), cpos, clen, ccap);
  }
}

// ===========================================================================
// framing: candidate links, runs, pointer jumping
// ===========================================================================
// little-endian int64 at byte offset p of the stream (buf 8-B aligned);
// never reads at or beyond B
__device__ __forceinline__ uint64_t ld_le64_b(const uint8_t *buf, uint64_t B, uint64_t p) {
  const uint64_t al = p & ~7ull;
  if (al + 16 <= B) {
    const uint64_t lo = *(const uint64_t *)(buf + al), hi = *(const uint64_t *)(buf + al + 8);
    const uint32_t sh = (uint32_t)(p & 7) * 8;
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  }
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i)
    if (p + i < B) v |= (uint64_t)buf[p + i] << (8 * i);
  return v;
}

// Candidate i -> its length L (the int64 prefix) and successor candidate
// (pos + 8 + L), grid-stride over the K candidates counted on the device.
// Also decides whether the candidates form ONE chain from byte 0 (the
// normal case: nxt[i] == i + 1 everywhere), so the pointer-jumping framing
// can be skipped, and records that chain's terminal offset q and the int64
// there; initialises the ReadAll reductions.
__global__ __launch_bounds__(256) void k_link(const uint8_t *__restrict__ buf, uint64_t B,
                                              const uint64_t *__restrict__ pos, uint64_t *__restrict__ len,
                                              uint64_t ccap, uint32_t *__restrict__ nxt, uint8_t *__restrict__ exc,
                                              Small *ds) {
  const uint64_t K = ds->total < ccap ? ds->total : ccap;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  if (g0 == 0) {
    ds->agg.first_fail = ~0ull;
    ds->agg.last_entry = -1;
    ds->agg.last_state = -1;
    ds->agg.first_meta = ~0ull;
    ds->pos0 = K ? pos[0] : ~0ull;
  }
  uint32_t irr = 0;
  for (uint64_t i = g0; i < K; i += stride) {
    const uint64_t p = pos[i];
    const uint64_t L = ld_le64_b(buf, B, p);
    len[i] = L;
    const uint64_t s = p + 8 + L;
    uint32_t r = EW_NIL;
    if (i + 1 < K) {
      const uint64_t p1 = pos[i + 1];
      if (p1 == s) {
        r = (uint32_t)(i + 1);
      } else if (p1 < s) {
        uint64_t lo = i + 2, hi = K;
        while (lo < hi) {
          const uint64_t mid = lo + ((hi - lo) >> 1);
          if (pos[mid] < s) lo = mid + 1; else hi = mid;
        }
        if (lo < K && pos[lo] == s) r = (uint32_t)lo;
      }
      if (r != i + 1) irr = 1;
    } else {   // the last candidate: terminal of the regular chain
      ds->q = s;
      ds->qlen = (s <= B && B - s >= 8) ? (int64_t)ld_le64_b(buf, B, s) : 0;
    }
    nxt[i] = r;
    exc[i] = (r != i + 1);
  }
  if (__ballot(irr) && (threadIdx.x & 63) == 0) atomicOr(&ds->irregular, 1u);
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

// Chain entries of the marked runs.  A chain segment's first run has its
// entry set by k_jstart; every later run is entered at its predecessor's
// link.  last_cand = the largest terminal candidate of the marked runs: the
// chain segments are marked in position order, so that is the terminal of
// the segment marked last (k_jstart resets it).
__global__ void k_entry(const uint32_t *__restrict__ E, const uint32_t *__restrict__ nxt,
                        const uint32_t *__restrict__ rs, const uint8_t *__restrict__ vis, uint32_t R,
                        uint32_t *__restrict__ entry, ChainInfo *ci) {
  uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= R) return;
  if (!vis[a]) return;
  uint32_t r = rs[a];
  if (r != EW_NIL) entry[r] = nxt[E[a]];
  else atomicMax(&ci->last_cand, E[a]);
}

// A chain segment starts at candidate `cand`: mark its run, entered there.
__global__ void k_jstart(const uint32_t *__restrict__ E, uint32_t R, uint32_t cand, uint8_t *__restrict__ vis,
                         uint32_t *__restrict__ entry, ChainInfo *ci) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t a = lower_bound_u32(E, R, cand);
  if (a < R) {
    vis[a] = 1;
    entry[a] = cand;
  }
  ci->last_cand = 0;
}

__global__ void k_member(const uint32_t *__restrict__ E, uint32_t R, const uint8_t *__restrict__ vis,
                         const uint32_t *__restrict__ entry, uint32_t K, uint8_t *__restrict__ on) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  uint32_t a = lower_bound_u32(E, R, i);
  on[i] = (a < R && vis[a] && i >= entry[a]) ? 1 : 0;
}

// ===========================================================================
// per-frame decode (walpb.Record, raftpb.Entry, raftpb.HardState) + verify
// ===========================================================================

// Stream prefix P(x) = lin(stream[0..x)) from the per-unit prefix and the
// super-piece lins of k_stream, in two phases so a caller can issue the loads
// (the unit's prefix, its 16 super-piece lins, the 256-B super-piece holding
// x) together with its own and do the arithmetic later: Horner over the whole
// super-pieces before x (S_256), then slicing-by-4 / byte steps over the bytes
// of x's super-piece before x.
struct PrefixIn {
  uint32_t pw, k, tail;
  uint4 vv[EW_VPU / 4];
  uint4 dd[EW_VPIECE / 16];
};
__device__ __forceinline__ void prefix_load(uint64_t x, const uint32_t *__restrict__ pwave,
                                            const uint32_t *__restrict__ v, const uint8_t *__restrict__ buf,
                                            PrefixIn &in) {
  const uint64_t w = x >> 12;
  const uint64_t x0 = x & ~(uint64_t)(EW_VPIECE - 1);
  in.k = (uint32_t)((x0 >> EW_VLOG) & (EW_VPU - 1));
  in.tail = (uint32_t)(x - x0);
  const uint4 *vq = (const uint4 *)(v + w * EW_VPU);
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) in.vv[q] = (4u * q < in.k) ? vq[q] : make_uint4(0, 0, 0, 0);
  const uint4 *dq = (const uint4 *)(buf + x0);
#pragma unroll
  for (int q = 0; q < EW_VPIECE / 16; ++q) in.dd[q] = (16u * q < in.tail) ? dq[q] : make_uint4(0, 0, 0, 0);
  in.pw = pwave[w];
}
__device__ __forceinline__ uint32_t prefix_finish(const PrefixIn &in, const uint32_t *t4, const uint32_t *svp) {
  const uint32_t k = in.k, tail = in.tail;
  uint32_t acc = in.pw;
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) {
    if (4u * q + 0 < k) acc = tab_apply(svp, acc) ^ in.vv[q].x;
    if (4u * q + 1 < k) acc = tab_apply(svp, acc) ^ in.vv[q].y;
    if (4u * q + 2 < k) acc = tab_apply(svp, acc) ^ in.vv[q].z;
    if (4u * q + 3 < k) acc = tab_apply(svp, acc) ^ in.vv[q].w;
  }
  const uint32_t nd = tail >> 2;
#pragma unroll
  for (int q = 0; q < EW_VPIECE / 16; ++q) {
    if (4u * q + 0 < nd) acc = step4_flat(t4, acc ^ in.dd[q].x);
    if (4u * q + 1 < nd) acc = step4_flat(t4, acc ^ in.dd[q].y);
    if (4u * q + 2 < nd) acc = step4_flat(t4, acc ^ in.dd[q].z);
    if (4u * q + 3 < nd) acc = step4_flat(t4, acc ^ in.dd[q].w);
  }
  // remaining 0..3 bytes live in dword nd
  const uint32_t rem = tail & 3;
  if (rem) {
    uint32_t wd = 0;
#pragma unroll
    for (int q = 0; q < EW_VPIECE / 16; ++q) {
      if ((nd >> 2) == (uint32_t)q) {
        const uint32_t s = nd & 3;
        wd = s == 0 ? in.dd[q].x : s == 1 ? in.dd[q].y : s == 2 ? in.dd[q].z : in.dd[q].w;
      }
    }
    for (uint32_t b = 0; b < rem; ++b) {
      acc = t4[(acc ^ wd) & 0xff] ^ (acc >> 8);
      wd >>= 8;
    }
  }
  return acc;
}
// Slicing-by-16 step over one 16-B chunk (t = 16 tables, t[k] = byte then k
// zero bytes): only the first dword's four lookups depend on c, so the
// dependent chain is one lookup level per 16 bytes.
__device__ __forceinline__ uint32_t step16(const uint32_t *t, uint32_t c, const uint4 &d) {
  const uint32_t x = c ^ d.x;
  const uint32_t a = t[15 * 256 + (x & 0xff)] ^ t[14 * 256 + ((x >> 8) & 0xff)] ^ t[13 * 256 + ((x >> 16) & 0xff)] ^
                     t[12 * 256 + (x >> 24)];
  const uint32_t b = t[11 * 256 + (d.y & 0xff)] ^ t[10 * 256 + ((d.y >> 8) & 0xff)] ^
                     t[9 * 256 + ((d.y >> 16) & 0xff)] ^ t[8 * 256 + (d.y >> 24)];
  const uint32_t e = t[7 * 256 + (d.z & 0xff)] ^ t[6 * 256 + ((d.z >> 8) & 0xff)] ^
                     t[5 * 256 + ((d.z >> 16) & 0xff)] ^ t[4 * 256 + (d.z >> 24)];
  const uint32_t f = t[3 * 256 + (d.w & 0xff)] ^ t[2 * 256 + ((d.w >> 8) & 0xff)] ^
                     t[1 * 256 + ((d.w >> 16) & 0xff)] ^ t[d.w >> 24];
  return a ^ b ^ e ^ f;
}
// prefix_finish with the slicing-by-16 tables t16 (the first 1024 entries are
// the slicing-by-4 tables)
__device__ __forceinline__ uint32_t prefix_finish16(const PrefixIn &in, const uint32_t *t16, const uint32_t *svp) {
  const uint32_t k = in.k, tail = in.tail;
  uint32_t acc = in.pw;
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) {
    if (4u * q + 0 < k) acc = tab_apply(svp, acc) ^ in.vv[q].x;
    if (4u * q + 1 < k) acc = tab_apply(svp, acc) ^ in.vv[q].y;
    if (4u * q + 2 < k) acc = tab_apply(svp, acc) ^ in.vv[q].z;
    if (4u * q + 3 < k) acc = tab_apply(svp, acc) ^ in.vv[q].w;
  }
  const uint32_t nq = tail >> 4;
  uint4 pc = in.dd[0];
#pragma unroll
  for (int q = 0; q < EW_VPIECE / 16; ++q) {
    if ((uint32_t)q < nq) acc = step16(t16, acc, in.dd[q]);
    if (q && (uint32_t)q == nq) pc = in.dd[q];
  }
  const uint32_t nd = (tail & 15) >> 2;
  if (nd > 0) acc = step4_flat(t16, acc ^ pc.x);
  if (nd > 1) acc = step4_flat(t16, acc ^ pc.y);
  if (nd > 2) acc = step4_flat(t16, acc ^ pc.z);
  uint32_t wd = nd == 0 ? pc.x : nd == 1 ? pc.y : nd == 2 ? pc.z : pc.w;
  for (uint32_t b = 0; b < (tail & 3); ++b, wd >>= 8) acc = t16[(acc ^ wd) & 0xff] ^ (acc >> 8);
  return acc;
}
__device__ __forceinline__ uint32_t prefix_at(uint64_t x, const uint32_t *__restrict__ pwave,
                                              const uint32_t *__restrict__ v, const uint8_t *__restrict__ buf,
                                              const uint32_t *t4, const uint32_t *svp) {
  PrefixIn in;
  prefix_load(x, pwave, v, buf, in);
  return prefix_finish(in, t4, svp);
}

// P(x) from the NEARER super-piece boundary (the fused frame pass): x in the
// upper half of its super-piece [x0, x1 = x0 + 256) takes P(x1) -- Horner over
// one more v value -- and steps BACK over stream[x, x1) with the inverse
// shift: P(x) = S_{x1-x}^-1(P(x1) ^ lin(stream[x, x1))) (lin(A||B) =
// S_|B|(lin A) ^ lin B).  At most 128 tail bytes instead of 255 (half the
// fetch and the slicing steps on average, 32 fewer VGPRs).  `inv`: nibble
// tables of S_{2^m}^-1, m = 0..6.
struct PrefixNear {
  uint32_t pw, nk, n, up, lead, slow;   // slow: x in the upper half of the stream's last, partial
                                        // super-piece (no next boundary): prefix_at instead
  uint4 vv[EW_VPU / 4];
  uint4 dd[8];   // n <= 128 either way: tail <= 128 forward, x1 - (x & ~15) <= 128 back
};
__device__ __forceinline__ void prefix_load_near(uint64_t x, uint64_t B, const uint32_t *__restrict__ pwave,
                                                 const uint32_t *__restrict__ v, const uint8_t *__restrict__ buf,
                                                 PrefixNear &in) {
  const uint64_t w = x >> 12;
  const uint64_t x0 = x & ~(uint64_t)(EW_VPIECE - 1);
  const uint32_t k = (uint32_t)((x0 >> EW_VLOG) & (EW_VPU - 1));
  const uint32_t tail = (uint32_t)(x - x0);
  in.up = tail > EW_VPIECE / 2 && x0 + EW_VPIECE <= B;
  in.slow = tail > EW_VPIECE / 2 && !in.up;
  in.nk = k + in.up;
  in.lead = (uint32_t)(x & 15);
  const uint64_t base = in.up ? (x & ~15ull) : x0;
  in.n = in.up ? (uint32_t)(x0 + EW_VPIECE - base) : (in.slow ? 0u : tail);   // bytes loaded from base
  const uint4 *vq = (const uint4 *)(v + w * EW_VPU);
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) in.vv[q] = (4u * q < in.nk) ? vq[q] : make_uint4(0, 0, 0, 0);
  const uint4 *dq = (const uint4 *)(buf + base);
#pragma unroll
  for (int q = 0; q < 8; ++q) in.dd[q] = (16u * q < in.n) ? dq[q] : make_uint4(0, 0, 0, 0);
  in.pw = pwave[w];
}
#ifndef EW_FR_ABL
#define EW_FR_ABL 0   // timing-only ablations of the frame pass (tools/): 1 no Horner over v, 2 no prefix tail,
                      // 4 no S_dlen in the checks; results are wrong
#endif
#ifndef EW_TAIL2
#define EW_TAIL2 1   // 0: the round-5 tails (forward / backward branches, binary inverse steps)
#endif
// x shifted by s bytes, -128 <= s <= 128 (s < 0: the inverse), with the
// EW_TAIL_TABS nibble tables (crc_math.h): two lookups rounds, a table base
// per lane (lanes going forward and back share the code)
__device__ __forceinline__ uint32_t tail_shift(const uint32_t *tt, bool neg, uint32_t u, uint32_t x) {
  const uint32_t *t1 = tt + ((neg ? 34u : 9u) + (u & 15)) * 128;
  const uint32_t *t2 = tt + ((neg ? 25u : 0u) + (u >> 4)) * 128;
  return nib_apply(t2, nib_apply(t1, x));
}
// The prefix tail from the Horner result acc at the boundary the load chose
// (prefix_load_near: x0 below x, or the next boundary x1 above it).  NCH: the
// chunks the load holds, BLK = 16 NCH bytes from its 16-B aligned base.
//
// EW_TAIL2 (round 6): one code path for both directions, off the Horner's
// chain.  c = lin of the whole BLK-byte block with the bytes outside the tail
// zeroed (chunk 0 below `lead` going back, the bytes from n on going forward;
// whole chunks past n come zero from the load) -- NCH full slicing-by-16
// steps from register 0, no per-byte steps, independent of acc.  Trailing
// zeros shift a lin (lin(D || 0^k) = S_k(lin D)) and leading ones do not, so
//   forward  [x0, x0 + n):  P(x) = S_n(acc) ^ S_{BLK-n}^-1(c)
//   back     [x, x1):       P(x) = S_{x1-x}^-1(acc) ^ S_{BLK-lead}^-1(c)
// (x1 - x = n - lead): two table shifts of acc after the Horner, where the
// branches stepped up to 8 chunks + 6 words/bytes forward or 7 inverse
// nibble rounds back -- and a wave holding lanes of both ran both.
template <int NCH, class PN>
__device__ __forceinline__ uint32_t prefix_near_tail(uint32_t acc, const PN &in, const uint32_t *t16,
                                                     const uint32_t *inv) {
#if EW_TAIL2
  constexpr uint32_t BLK = 16 * NCH;
  const uint32_t lo = in.up ? in.lead : 0u;   // chunk 0's bytes below lo are not the tail's
  const uint32_t r = in.n & 15, jp = in.n >> 4;   // going forward chunk jp holds r tail bytes
  uint32_t ml[4], mh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kl = (int)lo - 4 * i, kh = (int)r - 4 * i;   // bytes of word i below lo / below n
    ml[i] = kl <= 0 ? ~0u : kl >= 4 ? 0u : ~0u << (8 * kl);
    mh[i] = kh >= 4 ? ~0u : kh <= 0 ? 0u : (1u << (8 * kh)) - 1u;
  }
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    uint4 d = in.dd[q];
    if (q == 0) {
      d.x &= ml[0];
      d.y &= ml[1];
      d.z &= ml[2];
      d.w &= ml[3];
    }
    const bool pq = (uint32_t)q == jp;
    d.x &= pq ? mh[0] : ~0u;
    d.y &= pq ? mh[1] : ~0u;
    d.z &= pq ? mh[2] : ~0u;
    d.w &= pq ? mh[3] : ~0u;
    c = step16(t16, c, d);
  }
  const bool up = in.up;
  const uint32_t ua = up ? in.n - in.lead : in.n;
  const uint32_t uc = up ? BLK - in.lead : BLK - in.n;
  return tail_shift(inv, up, ua, acc) ^ tail_shift(inv, true, uc, c);
#else
  if (!in.up) {   // forward over the n bytes after x0
    const uint32_t nq = in.n >> 4;
    uint4 pc = in.dd[0];
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      if ((uint32_t)q < nq) acc = step16(t16, acc, in.dd[q]);
      if (q && (uint32_t)q == nq) pc = in.dd[q];
    }
    const uint32_t nd = (in.n & 15) >> 2;
    if (nd > 0) acc = step4_flat(t16, acc ^ pc.x);
    if (nd > 1) acc = step4_flat(t16, acc ^ pc.y);
    if (nd > 2) acc = step4_flat(t16, acc ^ pc.z);
    uint32_t wd = nd == 0 ? pc.x : nd == 1 ? pc.y : nd == 2 ? pc.z : pc.w;
    for (uint32_t b = 0; b < (in.n & 3); ++b, wd >>= 8) acc = t16[(acc ^ wd) & 0xff] ^ (acc >> 8);
    return acc;
  }
  // lin(stream[x, x1)) from register 0: chunk 0 from byte `lead` on, then whole chunks
  uint32_t c = 0;
  const uint32_t lead = in.lead;
  const uint32_t w0[4] = {in.dd[0].x, in.dd[0].y, in.dd[0].z, in.dd[0].w};
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    if (4 * j >= lead) {
      c = step4_flat(t16, c ^ w0[j]);
    } else if (4 * j + 4 > lead) {
      uint32_t t = w0[j] >> (8 * (lead & 3));
      for (uint32_t b = lead & 3; b < 4; ++b, t >>= 8) c = t16[(c ^ t) & 0xff] ^ (c >> 8);
    }
  }
  const uint32_t nq = in.n >> 4;   // in.n is a multiple of 16 here
#pragma unroll
  for (int q = 1; q < NCH; ++q)
    if ((uint32_t)q < nq) c = step16(t16, c, in.dd[q]);
  uint32_t x = acc ^ c;
  const uint32_t m = in.n - lead;   // x1 - x, 1..127
#pragma unroll
  for (int l = 0; l < 7; ++l)
    if ((m >> l) & 1) x = nib_apply(inv + l * 128, x);
  return x;
#endif
}
__device__ __forceinline__ uint32_t prefix_finish_near(const PrefixNear &in, const uint32_t *t16, const uint32_t *svp,
                                                       const uint32_t *inv) {
  uint32_t acc = in.pw;
  if (EW_FR_ABL & 2) return acc ^ in.vv[0].x ^ in.dd[0].y;
#pragma unroll
  for (int q = 0; q < EW_VPU / 4 && !(EW_FR_ABL & 1); ++q) {
    if (4u * q + 0 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].x;
    if (4u * q + 1 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].y;
    if (4u * q + 2 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].z;
    if (4u * q + 3 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].w;
  }
  return prefix_near_tail<8>(acc, in, t16, inv);
}

// The same at 128-B granularity (the frame pass on record-dense WALs, round
// 5): besides v[] the stream pass stored vh[], the lin of the FIRST 128-B
// half of every super-piece, so P at a mid boundary is S_128(P(super-piece
// start)) ^ vh -- the tail is at most 64 bytes forward or 64 stepped back
// (half the bytes, 4 chunks of registers instead of 8).
struct PrefixNearVH {
  uint32_t pw, nk, n, up, lead, slow, mid, vhv;   // mid: the boundary is a super-piece's 128-B mid point
  uint4 vv[EW_VPU / 4];
  uint4 dd[4];   // n <= 64
};
__device__ __forceinline__ void prefix_load_near_vh(uint64_t x, uint64_t B, uint32_t pw, const uint32_t *__restrict__ v,
                                                    const uint32_t *__restrict__ vh, const uint8_t *__restrict__ buf,
                                                    PrefixNearVH &in) {
  const uint64_t w = x >> 12;
  const uint64_t x0 = x & ~127ull;
  const uint32_t tail = (uint32_t)(x - x0);
  in.up = tail > 64 && x0 + 128 <= B;
  in.slow = tail > 64 && !in.up;
  const uint32_t rel = (uint32_t)((in.up ? x0 + 128 : x0) - (w << 12));   // the boundary in x's unit, 0..4096
  in.nk = rel >> 8;
  in.mid = (rel >> 7) & 1;
  in.lead = (uint32_t)(x & 15);
  const uint64_t base = in.up ? (x & ~15ull) : x0;
  in.n = in.up ? (uint32_t)(x0 + 128 - base) : (in.slow ? 0u : tail);
  const uint4 *vq = (const uint4 *)(v + w * EW_VPU);
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) in.vv[q] = (4u * q < in.nk) ? vq[q] : make_uint4(0, 0, 0, 0);
  in.vhv = in.mid ? vh[w * EW_VPU + in.nk] : 0u;
  const uint4 *dq = (const uint4 *)(buf + base);
#pragma unroll
  for (int q = 0; q < 4; ++q) in.dd[q] = (16u * q < in.n) ? dq[q] : make_uint4(0, 0, 0, 0);
  in.pw = pw;
}
__device__ __forceinline__ uint32_t prefix_finish_near_vh(const PrefixNearVH &in, const uint32_t *t16,
                                                          const uint32_t *svp, const uint32_t *inv,
                                                          const uint32_t *n128) {
  uint32_t acc = in.pw;
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) {
    if (4u * q + 0 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].x;
    if (4u * q + 1 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].y;
    if (4u * q + 2 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].z;
    if (4u * q + 3 < in.nk) acc = tab_apply(svp, acc) ^ in.vv[q].w;
  }
  if (in.mid) acc = nib_apply(n128, acc) ^ in.vhv;
  return prefix_near_tail<4>(acc, in, t16, inv);
}

// lin of the concatenation of every non-empty segment of bytes field fnum
// of a message pb_walk accepted (Go's `m.Data = append(m.Data, ...)` over
// repeats), the message read at stream offset base:
//   lin(A || B) = S_|B|(lin A) ^ lin B,  lin[s, e) = S_{e-s}(P(s)) ^ P(e).
// Every other field is stepped over as proto.Skip would (its extent is the
// one the walker consumed).  Rare: split fields only.
template <class P>
__device__ uint32_t bytes_field_lin(const P &p, int64_t l, uint32_t fnum, uint64_t base, const uint8_t *__restrict__ buf,
                                    const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                                    const uint32_t *t4, const uint32_t *svp, const uint32_t *__restrict__ g_shift) {
  int64_t i = 0;
  uint32_t lin = 0;
  while (i < l) {
    const int64_t at = i;
    uint64_t wire = 0;
    if (rd_varint(p, i, l, wire, 64)) break;
    if ((uint32_t)(wire >> 3) == fnum && (wire & 7) == 2) {
      uint64_t bl = 0;
      if (rd_varint(p, i, l, bl, 64)) break;
      const int64_t post = (int64_t)((uint64_t)i + bl);
      if (post > i) {
        const uint64_t s0 = base + (uint64_t)i, e0 = base + (uint64_t)post;
        lin = gshift_n(g_shift, e0 - s0, lin ^ prefix_at(s0, pwave, v, buf, t4, svp)) ^
              prefix_at(e0, pwave, v, buf, t4, svp);
      }
      i = post;
      continue;
    }
    int64_t skippy = 0;
    if (pb_skip(gptr(p) + at, l - at, skippy) || skippy <= 0) break;
    i = at + skippy;
  }
  return lin;
}

// ---- split byte fields: the side arena ------------------------------------
// A bytes field repeated with several non-empty segments is, in Go, their
// concatenation (`m.Data = append(m.Data, data[i:post]...)`, record.pb.go:112,
// raft.pb.go:254).  Such frames (crafted: etcd's encoder writes each field
// once) get the concatenation gathered into a ctx-owned side arena, and every
// view into it is an offset there.  ~0: no room (Small.ncatfail, cat_need:
// the host grows the arena and runs the call again).
__device__ __forceinline__ uint64_t cat_alloc(uint8_t *cat, uint64_t catcap, Small *ds, uint64_t n) {
  const uint64_t co = atomicAdd(&ds->cat_used, (unsigned long long)n);
  if (cat == nullptr || co + n > catcap) {
    atomicMax(&ds->cat_need, (unsigned long long)(co + n));
    atomicAdd(&ds->ncatfail, 1u);
    return ~0ull;
  }
  return co;
}
// Every non-empty segment of bytes field fnum of message m (l bytes), in
// order, to dst (one thread; rare).  kvar / kbytes: the message's varint /
// bytes fields (pb_each's wire-type rule).
__device__ __forceinline__ void cat_gather(uint8_t *dst, const uint8_t *m, int64_t l, uint32_t fnum, uint32_t kvar,
                                           uint32_t kbytes) {
  uint64_t w = 0;
  pb_each(m, l, fnum, kvar, kbytes, [&](bool b, uint64_t off, uint64_t len) {
    if (!b) return;
    for (uint64_t k = 0; k < len; ++k) dst[w + k] = m[off + k];
    w += len;
  });
}
// Entry.Data split inside an Entry message at m (l bytes): its concatenation
// (total bytes) to the side arena; edoff then indexes the arena (pad1 bit 1).
__device__ __forceinline__ void entry_data_cat(const uint8_t *m, int64_t l, uint64_t total, uint8_t *cat,
                                               uint64_t catcap, Small *ds, RecDesc &d) {
  const uint64_t co = cat_alloc(cat, catcap, ds, total);
  if (co == ~0ull) {
    d.sub_st = 48;
    return;
  }
  cat_gather(cat + co, m, l, 4, 0xeu, 0x10u);
  d.edoff = co;
  d.edlen = total;
  d.enil = 0;
  d.pad1 |= 2;
}
// The metadata / Entry / HardState of a Record whose Data is the n bytes at
// arena offset co (mustUnmarshalEntry / mustUnmarshalState, wal/decoder.go:61-77);
// the Entry's Data is then a range of the arena too.
__device__ __forceinline__ void decode_inner(const uint8_t *m, int64_t n, uint64_t co, uint8_t *cat,
                                             uint64_t catcap, Small *ds, RecDesc &d) {
  if (d.type == 2) {
    PbField e1, e2, e3, e4, e5;
    pbf_init(e1); pbf_init(e2); pbf_init(e3); pbf_init(e4); pbf_init(e5);
    int ur = 0;
    const int s2 = pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(m, n, e1, e2, e3, e4, e5, ur, nullptr,
                                                                          nullptr, 0);
    d.pad1 = (s2 == 0 && ur) ? 1 : 0;
    d.sub_st = s2;
    d.etype = (int32_t)(uint32_t)e1.v;
    d.f0 = e2.v;
    d.f1 = e3.v;
    if (e4.blen > 0) { d.edoff = co + (uint64_t)e4.boff; d.edlen = (uint64_t)e4.blen; d.enil = 0; d.pad1 |= 2; }
    if (s2 == 0 && e4.split) entry_data_cat(m, n, (uint64_t)e4.blen, cat, catcap, ds, d);
  } else if (d.type == 3) {
    PbField h1, h2, h3, h4, h5;
    pbf_init(h1); pbf_init(h2); pbf_init(h3); pbf_init(h4); pbf_init(h5);
    int ur = 0;
    const int s2 = pb_walk<PB_VAR64, PB_VAR64, PB_VAR64, PB_NONE, PB_NONE>(m, n, h1, h2, h3, h4, h5, ur, nullptr,
                                                                         nullptr, 0);
    d.pad1 = (s2 == 0 && ur) ? 1 : 0;
    d.sub_st = s2;
    d.f0 = h1.v; d.f1 = h2.v; d.f2 = h3.v;
  }
}

// General decode of frame r (any encoding the reference accepts): the
// gogoprotobuf walkers over an LDS copy of the frame head, and P at its frame
// start and data start:
//   Pd[r] = P(doff) = raw(P(off), frame header bytes)
// plus, for the last frame, P at its data end (the frame after it is not on
// the chain).  The frame head (80 bytes from the 16-B boundary below the
// frame start) is fetched with five vector loads and parsed out of LDS.
__device__ __forceinline__ void decode_general(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p, int64_t L,
                                               uint32_t r, uint32_t n, const uint32_t *__restrict__ pwave,
                                               const uint32_t *__restrict__ v, const uint32_t *s_t4,
                                               const uint32_t *s_svp, const uint32_t *__restrict__ g_shift,
                                               uint4 (&win)[5], RecDesc *__restrict__ rd,
                                               uint32_t *__restrict__ pfd, uint32_t *__restrict__ pfo,
                                               uint8_t *__restrict__ cat, uint64_t catcap, Small *ds) {
  const uint64_t p16 = p & ~15ull;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint64_t o = p16 + 16 * k;
    uint4 w;
    if (o + 16 <= B) {
      w = *(const uint4 *)(buf + o);
    } else {
      uint32_t x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = load_word_guarded(buf, B, o + 4 * j);
      w = make_uint4(x[0], x[1], x[2], x[3]);
    }
    win[k] = w;
  }
  const WinReader R{(const uint8_t *)&win[0] + (p - p16), (int64_t)(80 - (p - p16)), buf + p};
  RecDesc d;
  d.off = p;
  d.type = 0; d.crc = 0; d.chained = 0; d.st = 0; d.sub_st = 0;
  d.doff = p + 8; d.dlen = 0; d.dnil = 1;
  d.f0 = d.f1 = d.f2 = 0; d.edoff = 0; d.edlen = 0; d.enil = 1; d.etype = 0; d.pad1 = 0;
  PbField a1, a2, a3, a4, a5;
  pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
  int unrec;
  int st = pb_walk<PB_VAR64, PB_VAR32, PB_BYTES, PB_NONE, PB_NONE>(R + 8, L, a1, a2, a3, a4, a5, unrec,
                                                                   nullptr, nullptr, 0);
  d.type = (int64_t)a1.v;
  d.crc = (uint32_t)a2.v;
  if (a3.blen > 0) { d.doff = p + 8 + a3.boff; d.dlen = a3.blen; d.dnil = 0; }
  d.st = st;
  const bool split = st == 0 && a3.split;   // Data in several segments: their concatenation
  d.pad0 = split ? 1 : 0;
  if (split) {
    // the CRC over the concatenation: k_check's Update(seed, D) =
    // S_n(seed ^ ~0 ^ P(s)) ^ P(e) ^ ~0 with P(s) := 0, P(e) := lin(D)
    pfo[r] = prefix_at(p, pwave, v, buf, s_t4, s_svp);
    pfd[r] = 0;
    d.chained = bytes_field_lin(R + 8, L, 3, p + 8, buf, pwave, v, s_t4, s_svp, g_shift);
    // Go's Data is the concatenation (`m.Data = append(m.Data, ...)`,
    // record.pb.go:112): gathered into the side arena, and the metadata /
    // Entry / HardState decoded from it there
    const uint64_t co = cat_alloc(cat, catcap, ds, (uint64_t)a3.blen);
    if (co == ~0ull) {   // no room: left undecoded (the host grows the arena and runs the call again)
      d.sub_st = 48;
      rd[r] = d;
      return;
    }
    cat_gather(cat + co, buf + p + 8, L, 3, 0x6u, 0x8u);
    decode_inner(cat + co, (int64_t)a3.blen, co, cat, catcap, ds, d);
    d.pad0 = 2;
    if (d.type == 2) d.f2 = co; else d.edoff = co;   // rd_cat_off
    rd[r] = d;
    return;
  }
  if (st == 0) {
    const WinReader dp = R + (int64_t)(d.doff - p);
    if (d.type == 2) {           // entryType: mustUnmarshalEntry
      PbField e1, e2, e3, e4, e5;
      pbf_init(e1); pbf_init(e2); pbf_init(e3); pbf_init(e4); pbf_init(e5);
      int s2 = 0, ur = 0;
      if (!d.dnil)
        s2 = pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(dp, (int64_t)d.dlen, e1, e2, e3, e4, e5, ur,
                                                                       nullptr, nullptr, 0);
      d.pad1 = (s2 == 0 && ur) ? 1 : 0;   // Entry.XXX_unrecognized: returned through the side list
      d.sub_st = s2;
      d.etype = (int32_t)(uint32_t)e1.v;
      d.f0 = e2.v;                  // Term
      d.f1 = e3.v;                  // Index
      if (e4.blen > 0) { d.edoff = d.doff + e4.boff; d.edlen = e4.blen; d.enil = 0; }
      if (s2 == 0 && e4.split) entry_data_cat(buf + d.doff, (int64_t)d.dlen, (uint64_t)e4.blen, cat, catcap, ds, d);
    } else if (d.type == 3) {    // stateType: mustUnmarshalState
      PbField h1, h2, h3, h4, h5;
      pbf_init(h1); pbf_init(h2); pbf_init(h3); pbf_init(h4); pbf_init(h5);
      int s2 = 0, ur = 0;
      if (!d.dnil)
        s2 = pb_walk<PB_VAR64, PB_VAR64, PB_VAR64, PB_NONE, PB_NONE>(dp, (int64_t)d.dlen, h1, h2, h3, h4, h5, ur,
                                                                      nullptr, nullptr, 0);
      d.pad1 = (s2 == 0 && ur) ? 1 : 0;   // HardState.XXX_unrecognized: returned through the side list
      d.sub_st = s2;
      d.f0 = h1.v; d.f1 = h2.v; d.f2 = h3.v;
    }
  }
  // P at every frame start (the previous frame's data end, in the canonical
  // layout), and P at this frame's data start from it (header bytes only).
  const uint32_t Pfo = prefix_at(p, pwave, v, buf, s_t4, s_svp);
  pfo[r] = Pfo;
  if (st == 0 && d.type != 4 && d.dlen > 0) {
    uint32_t c = Pfo;
    const int64_t nh = (int64_t)(d.doff - p);
    for (int64_t j = 0; j < nh; ++j) c = s_t4[(c ^ R[j]) & 0xff] ^ (c >> 8);
    pfd[r] = c;
    if (r == n - 1 || d.doff + d.dlen != p + 8 + (uint64_t)L)
      d.chained = prefix_at(d.doff + d.dlen, pwave, v, buf, s_t4, s_svp);   // P(data end), used by k_check
  }
  rd[r] = d;
}

// The frames the canonical parser declined, grid-stride over the device-side
// count (rec_cand == nullptr: frame r is candidate r).
__global__ __launch_bounds__(256) void k_decode_slow(const uint8_t *__restrict__ buf, uint64_t B,
                         const uint64_t *__restrict__ pos, const uint32_t *__restrict__ rec_cand,
                         const uint32_t *__restrict__ slow, Small *dsw, const uint32_t *__restrict__ pwave,
                         const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                         const uint32_t *__restrict__ g_shift, RecDesc *__restrict__ rd, uint32_t *__restrict__ pfd,
                         uint32_t *__restrict__ pfo, uint32_t n_host, uint8_t *__restrict__ cat,
                         uint64_t catcap) {
  Small *ds = dsw;
  const uint32_t ns = ds->nslow;
  if (ns == 0) return;
  // frames on the chain: the host's count, or the device's candidate count (k_frame)
  const uint32_t n = n_host ? n_host : (uint32_t)ds->total;
  __shared__ uint32_t s_t4[1024];
  __shared__ uint32_t s_svp[1024];
  __shared__ uint4 s_win[256][5];
  stage_lds<256>(s_t4, 1024, [&](int i) { return g_slice[i]; });
  stage_lds<256>(s_svp, 1024, [&](int i) { return g_shift[EW_VLOG * 1024 + i]; });
  __syncthreads();
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += gridDim.x * blockDim.x) {
    const uint32_t r = slow[j];
    const uint64_t p = pos[rec_cand ? rec_cand[r] : r];
    decode_general(buf, B, p, (int64_t)ld_le64_b(buf, B, p), r, n, pwave, v, s_t4, s_svp, g_shift, s_win[threadIdx.x],
                   rd, pfd, pfo, cat, catcap, ds);
  }
}

// ---- frames that are not candidates ---------------------------------------
// The candidate filter only admits the canonical Record head (08 <type<0x80>
// 10), so a frame that fits in the stream but is not a candidate -- a
// corrupted tag / type byte, a type >= 0x80, a non-canonical encoding --
// ends the candidate chain.  decoder.decode still reads it (wal/decoder.go:
// 28-47): k_walk follows the true frame chain from there, one frame at a
// time, with the exact walkers (Record.Unmarshal, record.pb.go:43-136; the
// CRC from the stream prefixes; Entry / HardState Unmarshal), until it meets
// a candidate again (the candidate chain resumes there), the stream's end /
// a frame that does not fit (the terminal), or a frame that fails (ReadAll
// stops there: nothing after it can change the result).  The frames it
// passes are listed in xpos and decoded with the chain's other frames.

// Would ReadAll continue after the frame at x (length L, fits), given the
// previous frame's stored CRC as the running CRC (k_check's local rule)?
// *crc = this frame's stored CRC.  Rules ReadAll applies across frames
// (metadata equality, the ents index gap) are left to k_check / k_result:
// continuing past such a frame costs only walk steps.
__device__ bool walk_passes(const uint8_t *__restrict__ buf, uint64_t x, int64_t L, uint32_t seed,
                            const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                            const uint32_t *__restrict__ g_slice, const uint32_t *__restrict__ g_shift, uint32_t *crc) {
  const uint8_t *rb = buf + x + 8;
  PbField a1, a2, a3, a4, a5;
  pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
  int unrec = 0;
  const int st = pb_walk<PB_VAR64, PB_VAR32, PB_BYTES, PB_NONE, PB_NONE>(rb, L, a1, a2, a3, a4, a5, unrec, nullptr,
                                                                         nullptr, 0);
  *crc = (uint32_t)a2.v;
  if (st) return false;
  const int64_t type = (int64_t)a1.v;
  if (type == 4) return !(seed != 0 && *crc != seed);   // wal/wal.go:184-192
  uint32_t computed = seed;
  const uint32_t *svp = g_shift + EW_VLOG * 1024;
  if (a3.split) {   // Data = the concatenation of its segments
    const uint32_t lin = bytes_field_lin(rb, L, 3, x + 8, buf, pwave, v, g_slice, svp, g_shift);
    computed = gshift_n(g_shift, (uint64_t)a3.blen, seed ^ 0xffffffffu) ^ lin ^ 0xffffffffu;
  } else if (a3.blen > 0) {
    const uint64_t s = x + 8 + (uint64_t)a3.boff, e = s + (uint64_t)a3.blen;
    const uint32_t Ps = prefix_at(s, pwave, v, buf, g_slice, svp), Pe = prefix_at(e, pwave, v, buf, g_slice, svp);
    computed = gshift_n(g_shift, (uint64_t)a3.blen, seed ^ 0xffffffffu ^ Ps) ^ Pe ^ 0xffffffffu;
  }
  if (computed != *crc) return false;                   // walpb.ErrCRCMismatch
  // Data in several segments: the frame is listed and decoded from their
  // concatenation later (k_decode_slow); walking on past it costs only walk
  // steps when its Entry / HardState then fails (k_check finds the first failure)
  if (a3.split) return type == 1 || type == 2 || type == 3;
  if (type == 1) return true;
  if (type != 2 && type != 3) return false;             // unexpected block type
  if (a3.blen <= 0) return true;                        // Unmarshal(nil): the zero message
  const uint8_t *dp = rb + a3.boff;
  PbField e1, e2, e3, e4, e5;
  pbf_init(e1); pbf_init(e2); pbf_init(e3); pbf_init(e4); pbf_init(e5);
  int s2, ur = 0;
  if (type == 2)
    s2 = pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(dp, a3.blen, e1, e2, e3, e4, e5, ur, nullptr,
                                                                  nullptr, 0);
  else
    s2 = pb_walk<PB_VAR64, PB_VAR64, PB_VAR64, PB_NONE, PB_NONE>(dp, a3.blen, e1, e2, e3, e4, e5, ur, nullptr,
                                                                 nullptr, 0);
  return s2 == 0;   // XXX_unrecognized does not stop ReadAll
}

struct WalkOut {
  uint64_t x;         // where the walk ended
  uint64_t resume;    // the candidate at x (the candidate chain resumes there), ~0: none
  int32_t term;       // x is the terminal: EWAL_OK (clean end) or its class; -1: not a terminal
  int32_t stopped;    // the last listed frame fails: ReadAll stops there
  uint32_t n;         // frames listed in xpos
  uint32_t seed;      // the last listed frame's stored CRC
};

// One thread walks the frame chain from q.  The running CRC starts at the
// stored CRC of the frame before q: candidate pc's (EW_NIL: none, 0), or
// seed0 when has_seed (a walk continued after its list filled).
__global__ void k_walk(const uint8_t *__restrict__ buf, uint64_t B, uint64_t q, const uint64_t *__restrict__ cpos,
                       uint64_t K, uint32_t pc, int has_seed, uint32_t seed0, const uint32_t *__restrict__ pwave,
                       const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                       const uint32_t *__restrict__ g_shift, uint64_t *__restrict__ xpos, uint32_t xcap, WalkOut *o) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t seed = seed0;
  if (!has_seed) {
    seed = 0;
    if (pc != EW_NIL) {
      const uint64_t p = cpos[pc];
      PbField a1, a2, a3, a4, a5;
      pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
      int unrec = 0;
      (void)pb_walk<PB_VAR64, PB_VAR32, PB_BYTES, PB_NONE, PB_NONE>(buf + p + 8, (int64_t)ld_le64_b(buf, B, p), a1, a2,
                                                                    a3, a4, a5, unrec, nullptr, nullptr, 0);
      seed = (uint32_t)a2.v;
    }
  }
  WalkOut r;
  r.resume = ~0ull;
  r.term = -1;
  r.stopped = 0;
  uint64_t x = q;
  uint32_t n = 0;
  for (;;) {
    if (x == B) { r.term = EWAL_OK; break; }
    if (B - x < 8) { r.term = EWAL_ERR_UNEXPECTED_EOF; break; }
    const int64_t L = (int64_t)ld_le64_b(buf, B, x);
    const uint64_t rem = B - x - 8;
    if (L < 0) { r.term = EWAL_PANIC_NEG_LENGTH; break; }
    if ((uint64_t)L > rem) { r.term = rem == 0 ? EWAL_OK : EWAL_ERR_UNEXPECTED_EOF; break; }
    uint64_t lo = 0, hi = K;   // a candidate: the chain of candidates resumes here
    while (lo < hi) {
      const uint64_t mid = lo + ((hi - lo) >> 1);
      if (cpos[mid] < x) lo = mid + 1; else hi = mid;
    }
    if (lo < K && cpos[lo] == x) { r.resume = lo; break; }
    if (n == xcap) break;      // list full: the host continues from x
    xpos[n++] = x;
    uint32_t crc;
    const bool pass = walk_passes(buf, x, L, seed, pwave, v, g_slice, g_shift, &crc);
    seed = crc;
    x += 8 + (uint64_t)L;
    if (!pass) { r.stopped = 1; break; }
  }
  r.x = x;
  r.n = n;
  r.seed = seed;
  *o = r;
}

// The chain's frame positions when walked frames join the candidate chain:
// the nc chain candidates (cand list rc, or candidates 0..nc-1 when rc is
// null) merged with the nx walked frames (both ascending) -> fpos.
__global__ void k_fpos(const uint64_t *__restrict__ cpos, const uint32_t *__restrict__ rc, uint32_t nc,
                       const uint64_t *__restrict__ xpos, uint32_t nx, uint64_t *__restrict__ fpos) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nc) {
    const uint64_t p = cpos[rc ? rc[t] : t];
    uint32_t lo = 0, hi = nx;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (xpos[mid] < p) lo = mid + 1; else hi = mid;
    }
    fpos[t + lo] = p;
  } else if (t < nc + nx) {
    const uint32_t e = t - nc;
    const uint64_t p = xpos[e];
    uint32_t lo = 0, hi = nc;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (cpos[rc ? rc[mid] : mid] < p) lo = mid + 1; else hi = mid;
    }
    fpos[e + lo] = p;
  }
}

// Fresh ReadAll reductions before a frame list is decoded and checked again.
__global__ void k_reset_check(Small *ds) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ds->agg.first_fail = ~0ull;
  ds->agg.last_entry = -1;
  ds->agg.last_state = -1;
  ds->agg.first_meta = ~0ull;
  ds->nmeta = 0;
  ds->nslow = 0;
  ds->nsel3 = 0;
  ds->lastop = 0;
  ds->gapslow = 0;
  ds->nonmono = 0;
  ds->nunrec = 0;
  ds->irregular = 0;
  ds->segbad = 0;
  ds->spec_n = 0;
  ds->fc_done = 0;
  ds->fc.fail_inv = 0;
  ds->fc.meta_inv = 0;
  ds->fc.last_entry1 = 0;
  ds->fc.last_state1 = 0;
  ds->fc.rare = 0;
  ds->fc.last_chained = 0;
}

// ---- canonical fast path ---------------------------------------------------
// The frame head (80 bytes from the 16-B boundary below the frame start) in
// LDS, TRANSPOSED: dword k of thread t at w[k * 256] (w = s_win + t), so the
// bank of every read is t & 31 whatever offset each lane reads.
// (WS: the window's dword stride, the workgroup size)
template <int WS = 256>
__device__ __forceinline__ uint32_t win4(const uint32_t *w, int o) {
  const int k = o >> 2;
  return __builtin_amdgcn_alignbyte(w[(k + 1) * WS], w[k * WS], (uint32_t)(o & 3));
}
template <int WS = 256>
__device__ __forceinline__ uint64_t win8(const uint32_t *w, int o) {
  const int k = o >> 2;
  const uint32_t a = w[k * WS], b = w[(k + 1) * WS], c = w[(k + 2) * WS];
  const uint32_t sh = (uint32_t)(o & 3);
  return ((uint64_t)__builtin_amdgcn_alignbyte(c, b, sh) << 32) | __builtin_amdgcn_alignbyte(b, a, sh);
}
// tag byte + varint of at most 7 bytes at window offset o: returns the offset
// after the field, clears ok on a different tag, a longer varint or a field
// outside the window (the general walker then takes the frame).
template <int WS = 256>
__device__ __forceinline__ int pb_field_fast(const uint32_t *w, int o, uint32_t tag, uint64_t &v, bool &ok) {
  const int oc = o <= 71 ? o : 71;
  const uint64_t x = win8<WS>(w, oc);
  const uint64_t t = ~(x >> 8) & 0x0080808080808080ull;   // terminators among the 7 bytes after the tag
  const int nb = t ? (__builtin_ctzll(t) >> 3) + 1 : 8;
  uint64_t y = (x >> 8) & (nb >= 8 ? 0x00ffffffffffffffull : ((1ull << (8 * nb)) - 1));
  y = ((y & 0x7f007f007f007f00ull) >> 1) | (y & 0x007f007f007f007full);
  y = ((y & 0x3fff00003fff0000ull) >> 2) | (y & 0x00003fff00003fffull);
  y = ((y & 0x0fffffff00000000ull) >> 4) | (y & 0x000000000fffffffull);
  v = y;
  ok = ok && o <= 71 && (uint32_t)(x & 0xff) == tag && nb < 8;
  return o + 1 + nb;
}

// Canonical decode of the frame at p (int64 length L read from the window,
// so no earlier pass has to fetch it): canonical encodings -- Record {08 type
// 10 crc [1a len Data]}, Entry {08 type 10 term 18 index [22 len Data]},
// HardState {08 term 10 vote 18 commit}, every varint at most 7 bytes, the
// last field ending exactly at the message end -- are parsed with word
// operations; returns false for any other frame (the general walkers take
// it: exact gogoprotobuf semantics).  Then P at the frame start (Pfo) and at
// the data start (Pfd, when type != 4 and Data is not empty).  The frame
// head and prefix_at's operands are loaded together, one memory round trip.
// w: this thread's LDS window column (stride WS dwords).
struct NoOp {
  __device__ void operator()() const {}
};
// The frame's loads (head + prefix operands) and the decode from them are
// split so a caller can keep the next frame's loads in flight while it
// decodes this one (canon_issue / canon_finish); decode_canon runs both.
// NEAR: 0 prefix_load (the general path), 1 prefix_load_near (the frame
// pass), 2 prefix_load_near_vh (the frame pass at 128-B granularity)
template <int NEAR>
struct CanonLoad {
  uint4 hq[5];
  typename std::conditional<NEAR == 2, PrefixNearVH,
                            typename std::conditional<NEAR == 1, PrefixNear, PrefixIn>::type>::type pin;
};
template <int NEAR>
__device__ __forceinline__ void canon_issue(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p,
                                            const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                                            CanonLoad<NEAR> &ld) {
  const uint64_t p16 = p & ~15ull;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint64_t o = p16 + 16 * k;
    if (o + 16 <= B) {
      ld.hq[k] = *(const uint4 *)(buf + o);
    } else {
      uint32_t x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = load_word_guarded(buf, B, o + 4 * j);
      ld.hq[k] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  }
  static_assert(NEAR != 2, "the frame pass loads its own operands (fr_decode)");
  if constexpr (NEAR == 1) prefix_load_near(p, B, pwave, v, buf, ld.pin);
  else prefix_load(p, pwave, v, buf, ld.pin);
}
template <int WS, int NEAR>
__device__ __forceinline__ bool canon_finish(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p,
                                             const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                                             const uint32_t *s_t4, const uint32_t *s_svp, uint32_t *w, RecDesc &d,
                                             int64_t &L, uint32_t &Pfo, uint32_t &Pfd, bool noprefix,
                                             const uint32_t *s_inv, const CanonLoad<NEAR> &ld,
                                             const uint32_t *s_n128 = nullptr) {
  const uint64_t p16 = p & ~15ull;
  const auto &pin = ld.pin;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    w[(4 * k) * WS] = ld.hq[k].x; w[(4 * k + 1) * WS] = ld.hq[k].y;
    w[(4 * k + 2) * WS] = ld.hq[k].z; w[(4 * k + 3) * WS] = ld.hq[k].w;
  }
  const int base = (int)(p - p16);
  L = (int64_t)win8<WS>(w, base);
  const int64_t end = 8 + L;          // message end, relative to p
  bool ok = L >= 0 && L < (1ll << 40);
  uint64_t ty = 0, cr = 0, dl = 0;
  int o = pb_field_fast<WS>(w, base + 8, 0x08, ty, ok);
  o = pb_field_fast<WS>(w, o, 0x10, cr, ok);
  const bool hasd = ok && (int64_t)(o - base) < end;
  if (hasd) o = pb_field_fast<WS>(w, o, 0x1a, dl, ok);
  ok = ok && (hasd ? (end - (int64_t)(o - base) == (int64_t)dl) : ((int64_t)(o - base) == end));
  d.off = p;
  d.type = (int64_t)ty;
  d.crc = (uint32_t)cr;
  d.chained = 0; d.st = 0; d.sub_st = 0;
  d.doff = p + 8; d.dlen = 0; d.dnil = 1;
  d.f0 = d.f1 = d.f2 = 0; d.edoff = 0; d.edlen = 0; d.enil = 1; d.etype = 0; d.pad0 = 0; d.pad1 = 0;
  const int ho = o;                   // window offset of the data start
  if (hasd && dl > 0) { d.doff = p + (uint64_t)(o - base); d.dlen = dl; d.dnil = 0; }
  if (ok && !d.dnil && (d.type == 2 || d.type == 3)) {
    const int64_t eend = (int64_t)(ho - base) + (int64_t)dl;
    uint64_t f0 = 0, f1 = 0, f2 = 0;
    int e = pb_field_fast<WS>(w, ho, 0x08, f0, ok);
    e = pb_field_fast<WS>(w, e, 0x10, f1, ok);
    e = pb_field_fast<WS>(w, e, 0x18, f2, ok);
    if (d.type == 2) {                // Entry: Type, Term, Index [, Data]
      const bool hase = ok && (int64_t)(e - base) < eend;
      uint64_t el = 0;
      if (hase) e = pb_field_fast<WS>(w, e, 0x22, el, ok);
      ok = ok && (hase ? (eend - (int64_t)(e - base) == (int64_t)el) : ((int64_t)(e - base) == eend));
      d.etype = (int32_t)(uint32_t)f0;
      d.f0 = f1;
      d.f1 = f2;
      if (hase && el > 0) { d.edoff = p + (uint64_t)(e - base); d.edlen = el; d.enil = 0; }
    } else {                          // HardState: Term, Vote, Commit
      ok = ok && (int64_t)(e - base) == eend;
      d.f0 = f0; d.f1 = f1; d.f2 = f2;
    }
  }
  // P at the frame start even when the frame is not canonical: the frame
  // before it takes it as its P(data end) (a batched shard's torn last frame)
  if constexpr (NEAR == 2)   // (the frame pass: a slow position comes back as noprefix, fr_decode_slow)
    Pfo = noprefix ? pin.pw : prefix_finish_near_vh(pin, s_t4, s_svp, s_inv, s_n128);
  else if constexpr (NEAR == 1)
    Pfo = noprefix ? pin.pw
                   : (pin.slow ? prefix_at(p, pwave, v, buf, s_t4, s_svp) : prefix_finish_near(pin, s_t4, s_svp, s_inv));
  else Pfo = noprefix ? pin.pw : prefix_finish16(pin, s_t4, s_svp);
  if (!ok) return false;
  if (d.type != 4 && d.dlen > 0) {    // P(data start): the header bytes after P(frame start)
    uint32_t c = Pfo;
    const int nh = ho - base;
    int j = 0;
    for (; j + 4 <= nh; j += 4) c = step4_flat(s_t4, c ^ win4<WS>(w, base + j));
    uint32_t t = win4<WS>(w, base + j);
    for (; j < nh; ++j, t >>= 8) c = s_t4[(c ^ t) & 0xff] ^ (c >> 8);
    Pfd = c;
  }
  return true;
}
template <int WS, int NEAR = 0, class AfterIssue = NoOp>
__device__ __forceinline__ bool decode_canon(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p,
                                             const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                                             const uint32_t *s_t4, const uint32_t *s_svp, uint32_t *w, RecDesc &d,
                                             int64_t &L, uint32_t &Pfo, uint32_t &Pfd, bool noprefix = false,
                                             AfterIssue after_issue = AfterIssue(), const uint32_t *s_inv = nullptr) {
  CanonLoad<NEAR> ld;
  canon_issue<NEAR>(buf, B, p, pwave, v, ld);
  after_issue();   // the caller's stores: issued behind this frame's loads, so waiting for them never waits for those
  return canon_finish<WS, NEAR>(buf, B, p, pwave, v, s_t4, s_svp, w, d, L, Pfo, Pfd, noprefix, s_inv, ld);
}

// decode_canon for frame r of the general path: the descriptor and prefixes
// to HBM (rd, pfo, pfd; P(data end) in d.chained for the chain's last frame),
// or the frame to the slow list.  Returns L.
__device__ __forceinline__ int64_t decode_fast(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p, uint32_t r,
                                               bool last, const uint32_t *__restrict__ pwave,
                                               const uint32_t *__restrict__ v, const uint32_t *s_t4,
                                               const uint32_t *s_svp, uint32_t *w, RecDesc *__restrict__ rd,
                                               uint32_t *__restrict__ pfd, uint32_t *__restrict__ pfo,
                                               uint32_t *__restrict__ slow, Small *ds) {
  RecDesc d;
  int64_t L = 0;
  uint32_t Pfo = 0, Pfd = 0;
  if (!decode_canon<256>(buf, B, p, pwave, v, s_t4, s_svp, w, d, L, Pfo, Pfd)) {
    slow[atomicAdd(&ds->nslow, 1u)] = r;
    return L;
  }
  pfo[r] = Pfo;
  if (d.type != 4 && d.dlen > 0) {
    pfd[r] = Pfd;
    if (last) d.chained = prefix_at(d.doff + d.dlen, pwave, v, buf, s_t4, s_svp);   // P(data end)
  }
  rd[r] = d;
  return L;
}

// k_decode: the frames of a chain the host framed (frame r = candidate
// rec_cand[r], or candidate r when rec_cand is null).  Every list index is
// checked against the list's capacity (pcap, rccap) and every position
// against B: a frame list that breaks the host's invariant raises
// Small.errflag bit EW_ERR_LIST (the call fails with EWAL_E_INVAL) instead of
// reading out of bounds.
__global__ __launch_bounds__(256) void k_decode(const uint8_t *__restrict__ buf, uint64_t B,
                         const uint64_t *__restrict__ pos, uint64_t pcap, const uint32_t *__restrict__ rec_cand,
                         uint64_t rccap, uint32_t n,
                         const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                         const uint32_t *__restrict__ g_slice, const uint32_t *__restrict__ g_shift,
                         RecDesc *__restrict__ rd, uint32_t *__restrict__ pfd, uint32_t *__restrict__ pfo,
                         uint32_t *__restrict__ slow, Small *ds) {
  __shared__ uint32_t s_t4[16 * 256];   // slicing-by-16
  __shared__ uint32_t s_svp[1024];   // S_256 (prefix_at's Horner step)
  __shared__ uint32_t s_win[20 * 256];
  stage_lds<256>(s_t4, 16 * 256, [&](int i) { return g_slice[i]; });
  stage_lds<256>(s_svp, 1024, [&](int i) { return g_shift[EW_VLOG * 1024 + i]; });
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint64_t ix = rec_cand ? (r < rccap ? (uint64_t)rec_cand[r] : ~0ull) : (uint64_t)r;
  const uint64_t p = ix < pcap ? pos[ix] : ~0ull;
  if (p >= B) {
    atomicOr(&ds->errflag, EW_ERR_LIST);
    RecDesc d{};
    d.off = 0;
    d.type = 0;
    d.st = EWAL_ERR_UNEXPECTED_EOF;
    rd[r] = d;
    return;
  }
  decode_fast(buf, B, p, r, r == n - 1, pwave, v, s_t4, s_svp, s_win + threadIdx.x, rd, pfd, pfo, slow, ds);
}

// k_frame: framing and decode in one pass, speculating that the candidates
// form ONE chain from byte 0 (frame r = candidate r; the normal case).  Per
// candidate: its int64 length L (from the frame head it decodes anyway), the
// check that the next candidate starts at p + 8 + L (else the chain is
// irregular and the host redoes the framing by pointer jumping), the chain's
// terminal q and the int64 there, and the decode of the frame.  Grid-stride
// over the device-side candidate count; also initialises ReadAll's
// reductions.  Frames past rdcap (the descriptor capacity) are left to the
// host's retry with larger buffers.
__global__ __launch_bounds__(256) void k_frame(const uint8_t *__restrict__ buf, uint64_t B,
                         const uint64_t *__restrict__ pos, uint64_t ccap, uint64_t rdcap,
                         const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                         const uint32_t *__restrict__ g_slice, const uint32_t *__restrict__ g_shift,
                         RecDesc *__restrict__ rd, uint32_t *__restrict__ pfd, uint32_t *__restrict__ pfo,
                         uint32_t *__restrict__ slow, Small *ds, int dbg) {
  __shared__ uint32_t s_t4[16 * 256];   // slicing-by-16
  __shared__ uint32_t s_svp[1024];
  __shared__ uint32_t s_win[20 * 256];
  uint64_t K = ds->total;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  if (g0 == 0) {
    ds->agg.first_fail = ~0ull;
    ds->agg.last_entry = -1;
    ds->agg.last_state = -1;
    ds->agg.first_meta = ~0ull;
    ds->pos0 = K ? pos[0] : ~0ull;
  }
  if (K > ccap || K > rdcap || ds->novf) return;   // the host frames the slow way (larger buffers, k_rescan)
  stage_lds<256>(s_t4, 16 * 256, [&](int i) { return g_slice[i]; });
  stage_lds<256>(s_svp, 1024, [&](int i) { return g_shift[EW_VLOG * 1024 + i]; });
  __syncthreads();
  uint32_t irr = 0;
  // the candidate offsets of the NEXT iteration are loaded before this one's
  // frame head, so their latency hides behind it (one memory round trip per
  // frame instead of two)
  uint64_t p = g0 < K ? pos[g0] : 0, pn = g0 + 1 < K ? pos[g0 + 1] : 0;
  for (uint64_t r = g0; r < K; r += stride) {
    const uint64_t rn = r + stride;
    const uint64_t p2 = rn < K ? pos[rn] : 0, pn2 = rn + 1 < K ? pos[rn + 1] : 0;
    const int64_t L = decode_fast(buf, B, p, (uint32_t)r, r + 1 == K, pwave, v, s_t4, s_svp, s_win + threadIdx.x, rd,
                                  pfd, pfo, slow, ds);
    const uint64_t s = p + 8 + (uint64_t)L;
    if (r + 1 < K) {
      irr |= pn != s;
    } else {   // the last candidate: terminal of the regular chain
      ds->q = s;
      ds->qlen = (s <= B && B - s >= 8) ? (int64_t)ld_le64_b(buf, B, s) : 0;
    }
    p = p2;
    pn = pn2;
  }
  if (__ballot(irr) && (threadIdx.x & 63) == 0) atomicOr(&ds->irregular, 1u);
}

// k_check: the chained-CRC check of every frame (== the reference's running
// CRC up to its first failure), the Entry/HardState verdicts, the entry-op
// index-gap panic, ReadAll's reductions (first failure, last entry / state /
// op, first metadata), the per-workgroup op counts (k_opscan / k_opents) and
// the list of metadata frames k_result checks.
#define EW_GAP_BACK 16

// Decoupled look-back over per-workgroup counts (one wave): workgroup b
// publishes its count, then sums its predecessors' counts 64 at a time until
// it meets a published inclusive prefix, and publishes its own.  status[b] =
// epoch << 40 | flag << 32 | value (flag 1: the workgroup's count, 2: the
// inclusive prefix through it); an entry from an earlier call has another
// epoch and reads as not yet published.  Workgroups are dispatched in order
// (per XCD), so the lowest unfinished one is always resident and the waits
// drain; a spin budget reports EWAL_E_TIMEOUT instead of hanging.
__device__ __forceinline__ uint32_t lookback_count(unsigned long long *status, uint32_t b, uint32_t cnt,
                                                   uint32_t epoch, uint32_t *errflag) {
  const int lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)(epoch & 0xffffffu) << 40;
  if (b == 0) {
    if (lane == 0) __hip_atomic_store(&status[0], tag | (2ull << 32) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&status[b], tag | (1ull << 32) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t acc = 0;
  int64_t j = (int64_t)b - 1;
  uint32_t spins = 0;
  for (;;) {
    const int64_t idx = j - lane;
    unsigned long long sv = 0;
    int f = 2;                          // before workgroup 0: an inclusive prefix of 0
    if (idx >= 0) {
      sv = __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      f = ((sv >> 40) == (unsigned long long)(epoch & 0xffffffu)) ? (int)((sv >> 32) & 3) : 0;
    }
    const unsigned long long m2 = __ballot(f == 2), m0 = __ballot(f == 0);
    const int f2 = m2 ? __ffsll((long long)m2) - 1 : 64, f0 = m0 ? __ffsll((long long)m0) - 1 : 64;
    if (f2 < f0) {                      // lanes below f2 hold counts, lane f2 the inclusive prefix
      acc += __shfl(wave_incl_sum(lane <= f2 ? (uint32_t)sv : 0u), 63);
      break;
    }
    if (f0 < 64) {
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(errflag, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    acc += __shfl(wave_incl_sum((uint32_t)sv), 63);
    j -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(&status[b], tag | (2ull << 32) | (uint32_t)(acc + cnt), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return acc;
}
// last shard s in [a, b) with fs[s] <= r (fs ascending, fs[a] <= r)
__device__ __forceinline__ uint32_t shard_in(const uint32_t *__restrict__ fs, uint32_t a, uint32_t b, uint32_t r) {
  while (b - a > 1) {
    const uint32_t m = (a + b) >> 1;
    if (fs[m] <= r) a = m; else b = m;
  }
  return a;
}
__device__ __forceinline__ uint32_t shard_of(const uint32_t *__restrict__ fs, uint32_t ns, uint32_t r) {
  return shard_in(fs, 0, ns, r);
}

// SEG (ewal_readall_batch_device): the frames are the concatenation of many
// independent WALs (shards); frame r belongs to the last shard s with
// fs[s] <= r, every rule restarts at the shard's first frame (the running CRC
// at 0, the op list empty, ri = sg.ri[s]) and the reductions go to
// sg.sagg[s].  ents[j] keeps the global op order (a shard's ops are
// contiguous), with Data offsets relative to the shard.
template <bool SEG>
__global__ __launch_bounds__(1024) void k_check(const uint32_t *__restrict__ g_shift, RecDesc *__restrict__ rd,
                         uint32_t n, const uint32_t *__restrict__ pfd, const uint32_t *__restrict__ pfo, uint64_t ri,
                         unsigned long long *__restrict__ status, uint32_t epoch, uint32_t *__restrict__ wbase,
                         ewal_entry *__restrict__ ents, uint32_t *__restrict__ mlist, Small *ds, SegArgs sg,
                         const uint32_t *n_dev = nullptr) {
  // n_dev: launched before the host has seen k_frame's verdict (k_spec_gate
  // left the frame count there, 0 when the speculation failed); the grid is
  // sized for the descriptor capacity and the blocks past the frames leave
  if (n_dev) {
    n = *n_dev;
    if (blockIdx.x * blockDim.x >= n) return;
  }
  const uint32_t last_block = (n - 1) / blockDim.x;
  ReadAllAgg *agg = &ds->agg;
  __shared__ uint32_t s_wo[16];          // ops per wave
  __shared__ uint32_t s_base;            // ops before the workgroup
  __shared__ uint32_t s_sh[17 * 1024];   // S_{2^0} .. S_{2^16}
  __shared__ uint32_t s_red[5];          // block: last entry + 1, last state + 1, first metadata, first failure,
                                         //        last op + 1
  __shared__ uint32_t s_shr[2];          // SEG: shards of the workgroup's first and last frame
  stage_lds<1024>(s_sh, 17 * 1024, [&](int i) { return g_shift[i]; });
  if (threadIdx.x == 0) {
    s_red[0] = 0; s_red[1] = 0; s_red[2] = 0xffffffffu; s_red[3] = 0xffffffffu; s_red[4] = 0;
    if (SEG) {
      const uint32_t f0 = blockIdx.x * blockDim.x;
      s_shr[0] = shard_of(sg.fs, sg.ns, f0);
      s_shr[1] = shard_in(sg.fs, s_shr[0], sg.ns, min(f0 + blockDim.x, n) - 1);
    }
  }
  __syncthreads();
  const uint32_t rt = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = rt < n;
  const uint32_t r = live ? rt : n - 1;   // the whole block reaches the barrier below; writes masked
  // every load up front: the frame, its neighbours' CRC / offset, the prefixes
  const RecDesc d = rd[r];
  uint32_t sh = 0, lo = 0;                // the frame's shard and its first frame
  if (SEG) {   // usually one shard per workgroup: no search at all
    sh = s_shr[0] == s_shr[1] ? s_shr[0] : shard_in(sg.fs, s_shr[0], s_shr[1] + 1, r);
    lo = sg.fs[sh];
    ri = sg.ri[sh];
  }
  const uint32_t seed = r > lo ? rd[r - 1].crc : 0u;
  const uint64_t noff = r + 1 < n ? rd[r + 1].off : ~0ull;
  const uint32_t ps = pfd[r];
  const uint32_t pn = r + 1 < n ? pfo[r + 1] : 0u;
  int st = d.st;
  uint32_t chained = seed;
  if (st == 0) {
    if (d.type == 4) {                      // crcType: ReadAll's check, wal/wal.go:184-192
      if (seed != 0 && d.crc != seed) st = EWAL_ERR_WAL_CRC;
      chained = d.crc;
    } else {                                // decoder.decode: crc.Write(Data); Validate
      uint32_t computed;
      if (d.dlen == 0) {
        computed = seed;
      } else {
        const uint64_t e = d.doff + d.dlen;
        // P(data end) = P(next frame start) in the canonical layout (pfo[r+1]),
        // else k_decode left it in d.chained.  U(seed, D) = S_n(seed ^ ~0 ^ P(s)) ^ P(e) ^ ~0
        const uint32_t Pe = (noff == e && !d.pad0) ? pn : d.chained;
        uint32_t x = seed ^ 0xffffffffu ^ ps;
        uint64_t m = d.dlen;
        for (int lvl = 0; m; ++lvl, m >>= 1) {
          if (m & 1) x = lvl <= 16 ? tab_apply(s_sh + lvl * 1024, x) : gshift_pow2(g_shift, lvl, x);
        }
        computed = x ^ Pe ^ 0xffffffffu;
      }
      chained = computed;
      // a range split inside a file: frame 0's Validate is the caller's (its
      // chained value stays crc32.Update(0, Data) for ewal_copy_range_info)
      const bool defer0 = !SEG && r == 0 && ds->defer_first;
      if (computed != d.crc && !defer0) {
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
      } else if (d.sub_st == 48) {          // metadata Data in several segments
        st = EWAL_UNSUPPORTED_ENCODING;
      }
    }
  }
  // ReadAll's entry ops (wal/wal.go:170-176): an entry with Index >= ri is
  // appended at k = Index - ri, and ents[:k] panics when k > len(ents) =
  // k_prev + 1 (k_prev: the previous op's k; none: len 0).  Decided from the
  // decoded fields alone, as if every earlier frame verified: when one did
  // not, ReadAll stopped there and this frame's verdict is not the first
  // failure.  The previous op is found among the wave's lanes (ballot), else
  // by reading back at most EW_GAP_BACK earlier frames; farther -> the host's
  // list-based gap pass (ds->gapslow).
  const int lane = threadIdx.x & 63;
  const uint32_t r0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u);   // the wave's first frame
  const bool op = live && d.type == 2 && d.f1 >= ri;
  const unsigned long long mo = __ballot(op);
  const unsigned long long below = mo & ((1ull << lane) - 1ull);
  unsigned long long bsh = below;         // ops below in the same shard
  if (SEG && lo > r0) bsh = (lo - r0 >= 64) ? 0ull : below & ~((1ull << (lo - r0)) - 1ull);
  const uint64_t fprev = __shfl(d.f1, bsh ? 63 - __clzll((long long)bsh) : lane);   // every lane takes part
  if (op) {
    const uint64_t k = d.f1 - ri;
    bool has = bsh != 0;
    uint64_t kp = fprev - ri;
    uint32_t s2 = r0;           // the frames before the wave, back to the shard's first
    if (!has) {
      // SEG: a shard's first op usually follows its replayed-past entries
      // (Index < ri), so look back further before giving up (rare lanes)
      const int nback = SEG ? (1 << 16) : EW_GAP_BACK;
      for (int back = 0; back < nback && s2 > lo; ++back) {
        --s2;
        const int64_t t2 = rd[s2].type;
        const uint64_t i2 = rd[s2].f1;
        if (t2 == 2 && i2 >= ri) { kp = i2 - ri; has = true; break; }
      }
      if (!has && s2 > lo) atomicOr(&ds->gapslow, 1u);   // unresolved: k_gap decides
    }
    if (has || s2 <= lo) {
      if (has && k <= kp) atomicOr(&ds->nonmono, 1u);
      const bool gap = has ? (k > kp && k - kp > 1) : (k > 0);
      if (st == 0 && gap) st = EWAL_PANIC_INDEX_GAP;
    }
  }
  if (live) {
    rd[r].st = st;
    rd[r].chained = chained;
    if (d.type == 1 && st == 0) mlist[atomicAdd(&ds->nmeta, 1u)] = r;   // rare: one per WAL file
  }
  // One atomic per WORKGROUP and quantity (same-address atomics from every
  // wave serialise at the memory side): r grows with the lane and the wave,
  // so a wave's max is its highest set lane and its min its lowest.
  const unsigned long long me = __ballot(live && d.type == 2), ms = __ballot(live && d.type == 3),
                           mm = __ballot(live && d.type == 1 && d.dlen > 0), mf = __ballot(live && st != 0);
  // SEG: a workgroup inside one shard reduces through s_red like the single
  // WAL (thread 0 then updates sg.sagg); one that straddles shard
  // boundaries (rare) reduces per wave, or lane by lane where a boundary
  // lies inside the wave
  const bool wg1 = SEG && s_shr[0] == s_shr[1];
  if (SEG && !wg1) {
    const uint32_t s0 = __shfl(sh, 0);
    ShardAgg *A = sg.sagg + s0;
    if (__ballot(live && sh != s0) == 0) {
      if (lane == 0) {
        if (mf) atomicMin(&A->first_fail, (unsigned long long)(r0 + (uint32_t)(__ffsll((long long)mf) - 1)));
        if (me) atomicMax(&A->last_entry, (long long)(r0 + (uint32_t)(63 - __clzll((long long)me))));
        if (ms) atomicMax(&A->last_state, (long long)(r0 + (uint32_t)(63 - __clzll((long long)ms))));
        if (mm) atomicMin(&A->first_meta, (unsigned long long)(r0 + (uint32_t)(__ffsll((long long)mm) - 1)));
        if (mo) atomicMax(&A->lastop, r0 + (uint32_t)(63 - __clzll((long long)mo)) + 1u);
      }
    } else if (live) {   // a shard boundary inside the wave (rare): lane by lane
      A = sg.sagg + sh;
      if (st != 0) atomicMin(&A->first_fail, (unsigned long long)r);
      if (d.type == 2) atomicMax(&A->last_entry, (long long)r);
      if (d.type == 3) atomicMax(&A->last_state, (long long)r);
      if (d.type == 1 && d.dlen > 0) atomicMin(&A->first_meta, (unsigned long long)r);
      if (op) atomicMax(&A->lastop, r + 1u);
    }
  }
  if (lane == 0) {
    if (mf) atomicMin(&s_red[3], r0 + (uint32_t)(__ffsll((long long)mf) - 1));
    if (me) atomicMax(&s_red[0], r0 + (uint32_t)(63 - __clzll((long long)me)) + 1u);
    if (ms) atomicMax(&s_red[1], r0 + (uint32_t)(63 - __clzll((long long)ms)) + 1u);
    if (mm) atomicMin(&s_red[2], r0 + (uint32_t)(__ffsll((long long)mm) - 1));
    if (mo) atomicMax(&s_red[4], r0 + (uint32_t)(63 - __clzll((long long)mo)) + 1u);
    s_wo[threadIdx.x >> 6] = (uint32_t)__popcll(mo);
  }
  __syncthreads();
  if (threadIdx.x < 64) {   // wave 0: the workgroup's op base by decoupled look-back
    uint32_t cnt = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) cnt += s_wo[w];
    const uint32_t base = lookback_count(status, blockIdx.x, cnt, epoch, &ds->errflag);
    if (threadIdx.x == 0) {
      s_base = base;
      wbase[blockIdx.x] = base;   // k_opslist (rare paths) rebuilds ops / kk from it
      if (blockIdx.x == last_block) ds->nsel3 = base + cnt;
      if (s_red[0]) atomicMax(&agg->last_entry, (long long)(s_red[0] - 1));
      if (s_red[1]) atomicMax(&agg->last_state, (long long)(s_red[1] - 1));
      if (s_red[2] != 0xffffffffu) atomicMin(&agg->first_meta, (unsigned long long)s_red[2]);
      if (s_red[3] != 0xffffffffu) atomicMin(&agg->first_fail, (unsigned long long)s_red[3]);
      if (s_red[4]) atomicMax(&ds->lastop, s_red[4]);
      if (wg1) {
        ShardAgg *A = sg.sagg + s_shr[0];
        if (s_red[0]) atomicMax(&A->last_entry, (long long)(s_red[0] - 1));
        if (s_red[1]) atomicMax(&A->last_state, (long long)(s_red[1] - 1));
        if (s_red[2] != 0xffffffffu) atomicMin(&A->first_meta, (unsigned long long)s_red[2]);
        if (s_red[3] != 0xffffffffu) atomicMin(&A->first_fail, (unsigned long long)s_red[3]);
        if (s_red[4]) atomicMax(&A->lastop, s_red[4]);
        if (cnt) atomicMin(&A->ent_first, (unsigned long long)base);   // the workgroup's first op is op `base`
      }
    }
  }
  __syncthreads();
  if (op) {   // ents[j] = op j (exact when the ops' k are strictly increasing and gap-free,
              // otherwise the host's survivor pass rewrites ents)
    uint32_t j = s_base + (uint32_t)__popcll(below);
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int w = 0; w < 16; ++w) j += (w < wv) ? s_wo[w] : 0u;
    ewal_entry e;
    e.term = d.f0;
    e.index = d.f1;
    const bool side = (d.pad1 & 2) != 0;   // Data is a range of the side arena (split segments)
    e.data_off = (SEG && !side) ? d.edoff - sg.soff[sh] : d.edoff;
    e.data_len = d.edlen;
    e.type = d.etype;
    e.data_nil = side ? 2 : d.enil;
    ents[j] = e;
    if (SEG && !wg1 && bsh == 0) atomicMin(&sg.sagg[sh].ent_first, (unsigned long long)j);   // the shard's first op in the wave
    if (d.pad1 & 1) sg.ulist[atomicAdd(&ds->nunrec, 1u)] = make_uint2(r, j);   // rare: Entry.XXX_unrecognized
  }
}

// ops[j] = frame of op j, kk[j] = its k, from k_check's workgroup bases (the
// rare paths only: index gaps found far back, index rewinds).
__global__ __launch_bounds__(1024) void k_opslist(const RecDesc *__restrict__ rd, uint32_t n, uint64_t ri,
                                                  const uint32_t *__restrict__ wbase, uint32_t *__restrict__ ops,
                                                  uint64_t *__restrict__ kk) {
  __shared__ uint32_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t r = blockIdx.x * 1024 + tid;
  const bool live = r < n;
  const int64_t ty = live ? rd[r].type : 0;
  const uint64_t f1 = live ? rd[r].f1 : 0;
  const bool op = live && ty == 2 && f1 >= ri;
  const unsigned long long mo = __ballot(op);
  if (lane == 0) s_w[wv] = (uint32_t)__popcll(mo);
  __syncthreads();
  if (!op) return;
  uint32_t j = wbase[blockIdx.x] + (uint32_t)__popcll(mo & ((1ull << lane) - 1ull));
#pragma unroll
  for (int w = 0; w < 16; ++w) j += (w < wv) ? s_w[w] : 0u;
  ops[j] = r;
  kk[j] = f1 - ri;
}

// List-based gap check (the rare case where k_check could not find an op's
// predecessor nearby): op j needs k_j <= len(ents) = k_{j-1} + 1
// (wal/wal.go:173), over the op list k_opents wrote; frames k_check already
// failed keep their verdict.  Also flags k not strictly increasing.
__global__ void k_gap(RecDesc *__restrict__ rd, const uint32_t *__restrict__ ops, const uint64_t *__restrict__ kk,
                      Small *ds) {
  const uint32_t nops = ds->nsel3;
  uint32_t nm = 0;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nops; j += gridDim.x * blockDim.x) {
    const uint32_t r = ops[j];
    const uint64_t k = kk[j];
    bool gap;
    if (j == 0) {
      gap = k > 0;
    } else {
      const uint64_t kp = kk[j - 1];
      gap = (k > kp) && (k - kp > 1);
      if (k <= kp) nm = 1;
    }
    if (gap && rd[r].st == 0) {
      rd[r].st = EWAL_PANIC_INDEX_GAP;
      atomicMin(&ds->agg.first_fail, (unsigned long long)r);
    }
  }
  if (__ballot(nm) && (threadIdx.x & 63) == 0) atomicOr(&ds->nonmono, 1u);
}

// After k_frame: does the speculative frame pass hold (the host's test in
// readall_impl, made on the device so that k_check and k_result can be
// queued behind it without a host round trip)?  spec_n = frame count or 0;
// then Small -> host-mapped memory like k_export_small.
__global__ void k_spec_gate(Small *ds, uint64_t ccap, uint64_t rdcap, Small *h) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned long long K = ds->total;
  const bool ok = K && K <= ccap && K <= rdcap && !ds->novf && ds->pos0 == 0 && !ds->irregular;
  ds->spec_n = ok ? (uint32_t)K : 0u;
  *h = *ds;
}

// Small -> host-mapped pinned memory: a one-thread kernel is far cheaper
// than a device-to-host copy of a few hundred bytes.
__global__ void k_export_small(const Small *ds, Small *h) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *h = *ds;
}

// the handful of frames the host result needs, in one struct, written
// straight into host-mapped pinned memory
// One workgroup: first ReadAll's metadata rule, `metadata != nil &&
// !reflect.DeepEqual(metadata, rec.Data)` (wal/wal.go:178-183), over the
// metadata frames k_check listed (usually one per WAL file), then thread 0
// gathers the result.
__global__ __launch_bounds__(256) void k_result(const uint8_t *__restrict__ buf, RecDesc *__restrict__ rd,
                                                const uint32_t *__restrict__ mlist, uint32_t n, uint64_t ri, Small *ds,
                                                ResultDev *o, const uint32_t *n_dev, const uint8_t *__restrict__ cat) {
  if (n_dev) {   // speculative launch (see k_check): nothing to gather when it failed
    n = *n_dev;
    if (n == 0) return;
  }
  const uint32_t nm = ds->nmeta;
  const unsigned long long fm = ds->agg.first_meta;
  if (fm != ~0ull) {
    for (uint32_t i = threadIdx.x; i < nm; i += blockDim.x) {
      const uint32_t r = mlist[i];
      if (r <= fm) continue;
      RecDesc &d = rd[r];
      const RecDesc &m = rd[fm];
      bool eq = (d.dlen == m.dlen);
      // a split Data is its concatenation in the side arena
      const uint8_t *da = d.pad0 == 2 ? cat + rd_cat_off(d) : buf + d.doff;
      const uint8_t *ma = m.pad0 == 2 ? cat + rd_cat_off(m) : buf + m.doff;
      for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = da[k] == ma[k];
      if (!eq) {
        d.st = EWAL_ERR_METADATA_CONFLICT;
        atomicMin(&ds->agg.first_fail, (unsigned long long)r);
      }
    }
  }
  __threadfence();
  __syncthreads();
  if (threadIdx.x != 0) return;
  const ReadAllAgg g = ds->agg;
  o->agg = g;
  o->nops = ds->nsel3;
  o->nonmono = ds->nonmono;
  o->klast = ds->lastop ? rd[ds->lastop - 1].f1 - ri : 0;   // len(ents) - 1
  o->nslow = ds->nslow;
  o->gapslow = ds->gapslow;
  o->errflag = ds->errflag;
  o->nunrec = ds->nunrec;
  o->cat_used = ds->cat_used;
  o->cat_need = ds->cat_need;
  o->ncatfail = ds->ncatfail;
  if (g.first_fail < n) o->fail = rd[g.first_fail];
  if (g.last_entry >= 0) o->lastent = rd[g.last_entry];
  if (n) o->last = rd[n - 1];
  if (g.first_meta != ~0ull) o->md = rd[g.first_meta];
  if (g.last_state >= 0) o->sd = rd[g.last_state];
}

// ---- batched ReadAll over concatenated shards (ewal_readall_batch_device) --
// Every shard is an independent WAL byte stream (one raft group's
// names[nameIndex:], wal/wal.go:126-134) and the batch is their
// concatenation, so the frame chain of the batch runs through every shard
// when each one ends on a frame boundary -- which k_shard_start confirms
// (otherwise the host verifies the shards one by one).

// fs[s] = first frame at or after the shard's first byte; a non-empty shard
// must start exactly on a frame.  Also initialises the per-shard reductions.
__global__ void k_shard_start(const RecDesc *__restrict__ rd, uint32_t n, const uint64_t *__restrict__ soff,
                              uint32_t ns, uint32_t *__restrict__ fs, ShardAgg *__restrict__ sagg, Small *ds) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > ns) return;
  if (s == ns) {
    fs[ns] = n;
    return;
  }
  const uint64_t o = soff[s];
  uint32_t a = 0, b = n;
  while (a < b) {
    const uint32_t m = (a + b) >> 1;
    if (rd[m].off < o) a = m + 1; else b = m;
  }
  fs[s] = a;
  if (soff[s + 1] > o && (a >= n || rd[a].off != o)) atomicOr(&ds->segbad, 1u);
  ShardAgg g;
  g.first_fail = ~0ull;
  g.last_entry = -1;
  g.last_state = -1;
  g.first_meta = ~0ull;
  g.ent_first = ~0ull;
  g.lastop = 0;
  g.bad = 0;
  g.term1 = 0;
  g.term_st = 0;
  g.term_off = 0;
  sagg[s] = g;
}

// ReadAll's metadata rule per shard (wal/wal.go:178-183), over the metadata
// frames k_check<true> listed.
__global__ void k_meta_batch(const uint8_t *__restrict__ buf, RecDesc *__restrict__ rd,
                             const uint32_t *__restrict__ mlist, const Small *ds, SegArgs sg) {
  const uint32_t nm = ds->nmeta;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nm; i += gridDim.x * blockDim.x) {
    const uint32_t r = mlist[i];
    const uint32_t s = shard_of(sg.fs, sg.ns, r);
    const unsigned long long fm = sg.sagg[s].first_meta;
    if (fm == ~0ull || r <= fm) continue;
    RecDesc &d = rd[r];
    const RecDesc &m = rd[fm];
    bool eq = (d.dlen == m.dlen);
    for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = buf[d.doff + k] == buf[m.doff + k];
    if (!eq) {
      d.st = EWAL_ERR_METADATA_CONFLICT;
      atomicMin(&sg.sagg[s].first_fail, (unsigned long long)r);
    }
  }
}

// One thread per shard: its ReadAll result (the same assembly as the host's
// for one WAL, ewal_api.hip readall_impl), ordinals and offsets relative to
// the shard.  Every shard ends on a frame boundary here (k_shard_start), so
// its terminal is a clean io.EOF.
__global__ void k_result_batch(const RecDesc *__restrict__ rd, SegArgs sg, ewal_result *__restrict__ out,
                               unsigned long long *__restrict__ ent_first) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= sg.ns) return;
  const ShardAgg A = sg.sagg[s];
  const uint32_t f0 = sg.fs[s], f1 = sg.fs[s + 1];
  const uint64_t so = sg.soff[s], ri = sg.ri[s];
  ewal_result o;
  memset(&o, 0, sizeof(o));
  o.fail_record = -1;
  o.fail_offset = -1;
  o.metadata_off = -1;
  o.n_records = (int64_t)(f1 - f0);
  o.n_candidates = (int64_t)(f1 - f0);
  o.n_runs = 1;
  unsigned long long ef = 0;
  if (A.first_fail != ~0ull) {
    const RecDesc &f = rd[A.first_fail];
    o.status = f.st;
    o.fail_record = (int64_t)(A.first_fail - f0);
    o.fail_offset = (int64_t)(f.off - so);
    o.n_records = o.fail_record;
    if (f.st == EWAL_ERR_UNEXPECTED_TYPE) o.detail = f.type;
    if (f.st == EWAL_PANIC_INDEX_GAP) o.detail = (int64_t)f.f1;
  } else {
    const uint64_t enti = A.last_entry >= 0 ? rd[A.last_entry].f1 : 0;
    o.enti = enti;
    if (enti < ri) {
      o.status = EWAL_ERR_INDEX_NOT_FOUND;
    } else if (f1 > f0) {
      o.last_crc = rd[f1 - 1].chained;
      if (A.first_meta != ~0ull) {
        o.metadata_off = (int64_t)(rd[A.first_meta].doff - so);
        o.metadata_len = (int64_t)rd[A.first_meta].dlen;
      }
      if (A.last_state >= 0) {
        const RecDesc &sd = rd[A.last_state];
        o.has_state = 1;
        o.state_term = sd.f0;
        o.state_vote = sd.f1;
        o.state_commit = sd.f2;
      }
      // ops strictly increasing and gap-free here (else the host falls back)
      o.n_ents = A.lastop ? (int64_t)(rd[A.lastop - 1].f1 - ri + 1) : 0;
      ef = o.n_ents ? A.ent_first : 0;
    }
  }
  out[s] = o;
  ent_first[s] = ef;
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
    e.data_nil = (d.pad1 & 2) ? 2 : d.enil;   // 2: a range of the side arena
    ents[k] = e;
  }
}

// XXX_unrecognized of listed Entry / HardState frames (rare): PASS 0 sizes
// (the unknown fields the walker steps over, in order), PASS 1 copies them to
// arena + off -- Go's `m.XXX_unrecognized = append(m.XXX_unrecognized,
// data[iNdEx:iNdEx+skippy]...)` (raft/raftpb/raft.pb.go:270, :697).
template <int PASS>
__global__ void k_unrec(const uint8_t *__restrict__ buf, const RecDesc *__restrict__ rd, UnrecItem *__restrict__ it,
                        uint32_t m, uint8_t *__restrict__ arena, const uint8_t *__restrict__ cat) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const RecDesc d = rd[it[i].r];
  const uint8_t *dp = d.pad0 == 2 ? cat + rd_cat_off(d) : buf + d.doff;   // a split Data: its concatenation
  uint64_t tot = 0;
  uint8_t *dst = PASS ? arena + it[i].off : nullptr;
  auto unk = [&](int64_t a, int64_t b) {
    if (PASS)
      for (int64_t k = a; k < b; ++k) dst[tot + (uint64_t)(k - a)] = dp[k];
    tot += (uint64_t)(b - a);
  };
  PbField f1, f2, f3, f4, f5;
  pbf_init(f1); pbf_init(f2); pbf_init(f3); pbf_init(f4); pbf_init(f5);
  int ur = 0;
  if (d.type == 2)
    (void)pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(dp, (int64_t)d.dlen, f1, f2, f3, f4, f5, ur, nullptr,
                                                                   nullptr, 0, unk);
  else
    (void)pb_walk<PB_VAR64, PB_VAR64, PB_VAR64, PB_NONE, PB_NONE>(dp, (int64_t)d.dlen, f1, f2, f3, f4, f5, ur, nullptr,
                                                                  nullptr, 0, unk);
  if (!PASS) it[i].len = tot;
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

// What one rank's range of ONE WAL split by file contributes to the joined
// verdict (ewal_copy_range_info, etcd_amd/shard.py split_verdict): the first
// metadata frame (any Data, then non-nil Data), the first / last entry frame,
// the last entry op (Index >= ri, wal/wal.go:171) and the least Entry.Index,
// over the chain's frames.  Maxima are folded as frame + 1 (0: none).
struct RangeDev {
  unsigned long long md_first, md_value, ent_first, min_index;   // min (~0: none)
  unsigned long long ent_last1, op_last1, st_last1;              // max (0: none)
};
__global__ void k_range_info(const RecDesc *__restrict__ rd, uint32_t n, uint64_t ri, RangeDev *o) {
  unsigned long long mf = ~0ull, mv = ~0ull, ef = ~0ull, mi = ~0ull, el = 0, ol = 0, sl = 0;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const RecDesc &d = rd[r];
    if (d.type == 1) {
      mf = min(mf, (unsigned long long)r);
      if (!d.dnil && d.dlen) mv = min(mv, (unsigned long long)r);
    } else if (d.type == 2) {
      ef = min(ef, (unsigned long long)r);
      el = max(el, (unsigned long long)r + 1);
      if (d.f1 >= ri) ol = max(ol, (unsigned long long)r + 1);
      mi = min(mi, (unsigned long long)d.f1);
    } else if (d.type == 3) {
      sl = max(sl, (unsigned long long)r + 1);
    }
  }
  if (sl) atomicMax(&o->st_last1, sl);
  if (mf != ~0ull) atomicMin(&o->md_first, mf);
  if (mv != ~0ull) atomicMin(&o->md_value, mv);
  if (ef != ~0ull) atomicMin(&o->ent_first, ef);
  if (mi != ~0ull) atomicMin(&o->min_index, mi);
  if (el) atomicMax(&o->ent_last1, el);
  if (ol) atomicMax(&o->op_last1, ol);
}

__global__ void k_reverse_u64(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint32_t n) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) out[n - 1 - j] = in[j];
}

// P(x) for one x (pkg/crc digest over a whole device buffer).
// ---- ONE WAL split inside a file (ewal_range_probe) -------------------------
// The first frame-start candidate at or after `from` (the exact test of
// k_stream / k_cand: int64 length L in [4, B-p-8], the canonical Record head
// 08 <type<0x80> 10, record.pb.go:175-196), one position per thread -> the
// minimum in *pos (~0: none in the window).
__global__ void k_probe_cand(const uint8_t *__restrict__ buf, uint64_t B, uint64_t from, uint64_t end,
                             uint32_t align, unsigned long long *pos) {
  for (uint64_t p = from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < end;
       p += (uint64_t)gridDim.x * blockDim.x) {
    if ((p & (align - 1)) || p + 11 > B || buf[p + 8] != 0x08 || buf[p + 9] >= 0x80 || buf[p + 10] != 0x10) continue;
    const int64_t L = (int64_t)ld_le64_b(buf, B, p);
    if (L >= 4 && (uint64_t)L <= B - p - 8) atomicMin(pos, (unsigned long long)p);
  }
}
// From that candidate along the frame links (decoder.decode's framing,
// walpb.Record.Unmarshal, wal/decoder.go:28-47): the Index of the first entry
// record within `maxf` frames (mustUnmarshalEntry, raft.pb.go:170-277), for
// the range's w.ri.  out[0] = the candidate (or -1), out[1] = the Index (-1:
// none found).
__global__ void k_probe_walk(const uint8_t *__restrict__ buf, uint64_t B, const unsigned long long *pos,
                             uint32_t maxf, long long *out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned long long p0 = *pos;
  out[0] = p0 == ~0ull ? -1ll : (long long)p0;
  out[1] = -1;
  uint64_t p = p0;
  for (uint32_t f = 0; p0 != ~0ull && f < maxf; ++f) {
    if (p + 8 > B) break;
    const int64_t L = (int64_t)ld_le64_b(buf, B, p);
    if (L < 0 || (uint64_t)L > B - p - 8) break;
    PbField a1, a2, a3, a4, a5;
    pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
    int ur = 0;
    if (pb_walk<PB_VAR64, PB_VAR32, PB_BYTES, PB_NONE, PB_NONE>(buf + p + 8, L, a1, a2, a3, a4, a5, ur, nullptr,
                                                                nullptr, 0) != 0 || a3.split)
      break;
    if (a1.v == 2 && a3.blen > 0) {
      PbField e1, e2, e3, e4, e5;
      pbf_init(e1); pbf_init(e2); pbf_init(e3); pbf_init(e4); pbf_init(e5);
      if (pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(buf + p + 8 + a3.boff, a3.blen, e1, e2, e3, e4,
                                                                   e5, ur, nullptr, nullptr, 0) == 0)
        out[1] = (long long)e3.v;
      break;
    }
    p += 8 + (uint64_t)L;
  }
}

__global__ void k_prefix_one(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pwave,
                             const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                             const uint32_t *__restrict__ g_shift, uint64_t x, uint32_t *out) {
  if (threadIdx.x == 0) *out = prefix_at(x, pwave, v, buf, g_slice, g_shift + EW_VLOG * 1024);
}
