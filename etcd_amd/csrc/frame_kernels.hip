// frame_kernels.hip -- the frame pass after the stream pass: ONE kernel
// (k_frames) plus a seam pass (k_frames_seam) and the result gathers.
//
// Reference: (*WAL).ReadAll wal/wal.go:164-216, decoder.decode
// wal/decoder.go:28-47, walpb.Record.Unmarshal wal/walpb/record.pb.go:43-136,
// raftpb.Entry / HardState.Unmarshal raft/raftpb/raft.pb.go:170-277, 618-704.
//
// k_stream leaves, per 4 KiB unit, the lins of its 16 super-pieces (v[]) and
// the 64-B pieces its branch-free filter flagged (hmask).  k_frames takes the
// stream in TILES of TU = 2^TSH units (16, 64 or 256), one wave per tile:
//   A. the tile's unit lins (Horner over v[]) and their wave scan give P at
//      every unit start RELATIVE TO THE TILE START (Pl) -- no global prefix
//      scan: a record's check needs lin(Data) = S_n(P(s)) ^ P(e), the same for
//      any reference point; a record whose Data runs from tile a into tile b
//      takes lin[s, e) = S_{e-s}(Pl_a(s)) ^ S_{e-ts_b}(lin[ts_a, ts_b)) ^
//      Pl_b(e) in the seam pass (lin[ts_a, ts_b) from the tiles' aggregates);
//   B. the flagged pieces in rounds of 64, one per lane: each lane loads its
//      piece (64 B, +16 B when its last dword group was flagged) and runs the
//      exact frame-start tests -- the candidates;
//   C. the candidates in rounds of 63, one per lane (lane 0 holds the frame
//      carried from the previous round, whose check waited for its
//      successor): the canonical decode (the head and the prefix tail come
//      from the lines B just fetched: L2 hits), P at the frame and data
//      starts, the link to the successor, the chained-CRC check against the
//      predecessor's stored CRC, ReadAll's rules and the entry op stored at
//      ents[Index - ri].
// B runs one piece round ahead of C, so frame rounds stay full across piece
// rounds.  A tile's first and last frames (their neighbours live in other
// tiles) go to its FrTile for k_frames_seam.  Reductions are keyed by stream
// POSITION, not frame ordinal: ordinals are recovered only where a verdict
// names a frame (fr_ordinal: candidates of the tiles before, of the tile's
// units before, and an exact recount inside one unit).
//
// What the canonical pass does not decide -- a candidate chain broken by a
// false candidate, a non-canonical encoding, an index rewind, a record
// spanning more than FR_SCAN tiles, a whole frame after the chain's end that
// the filter did not admit -- sets Small.irregular / Small.fc.rare
// (single WAL) or ShardPos.bad (batch), and the host runs the general path
// over the same stream pass (ewal_api.hip); nothing is guessed.

#ifndef FR_HORNER_NIB
#define FR_HORNER_NIB 1    // phase A's Horner steps through the S_256 nibble tables (no bank conflicts)
#endif
#ifndef FR_DLEN2
#define FR_DLEN2 1         // the checks' S_dlen: its low 12 bits in three table rounds
#endif
#ifndef FR_COMPOSE_W
#define FR_COMPOSE_W 1     // fr_result's record composed by a wave (thread 0 alone: ~6 K cycles)
#endif
#ifndef FR_THREADS
#define FR_THREADS 768
#endif
#ifndef EW_ENTS_SC1
#define EW_ENTS_SC1 0      // A/B: the entry ops' ents slots stored sc1 (1: batch, 2: single WAL too)
#endif
#ifndef EW_FR_SC1
#define EW_FR_SC1 0        // A/B: the per-unit pl / ucb stored sc1
#endif
__device__ __forceinline__ void fr_st32(uint32_t *p, uint32_t x) {
  if (EW_FR_SC1) __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = x;
}
#define FR_WAVES (FR_THREADS / 64)
#define FR_NIB 20          // S_{2^0} .. S_{2^19} as nibble tables
#define FR_SCAN 4096       // tiles the seam pass scans for a tile's neighbouring frame

// Per tile: what k_frames_seam needs of its first and last frames, its entry
// ops and (single WAL) its reductions.  Positions are stream offsets.
struct FrTile {
  uint32_t count;          // candidates (frames) starting in the tile
  uint32_t agg;            // lin of the tile's bytes (zero-extended at the stream end)
  uint64_t p0, pz, sz;     // first frame start; last frame start and end (p + 8 + L)
  uint32_t pfo0;           // P(p0), tile-local
  uint32_t crcz;           // the last frame's stored CRC (the next tile's seed)
  int32_t type0, typez;
  uint32_t crc0, pfd0, pe0;   // the first frame's check operands (pe0: FRT_PE0)
  uint32_t seedz, pfdz;       // the last frame's (seedz: FRT_SEEDZ)
  uint32_t flags;
  uint32_t peB;            // the stream's last tile (FRT_PEB): P at the stream end, tile-local
  uint64_t dlen0, dlenz;
  // entry ops
  uint32_t nops, seam;     // seam: the gap rule for the tile's first op is the seam pass's
  uint64_t first_index, last_index;
  uint64_t firstop_p, lastop_p;
  // reductions (single WAL), positions
  unsigned long long fail;        // min (p << 8 | status), ~0
  uint64_t last_entry1, last_state1;   // 1 + position (max), 0: none
  uint64_t meta0;          // first metadata frame with non-empty Data, ~0
};
#define FRT_PE0 1u         // pe0 holds the first frame's P(data end) (its successor is in the tile)
#define FRT_SEEDZ 2u       // seedz holds the last frame's seed (a predecessor in the tile, or a shard start)
#define FRT_T0 4u          // the first frame's seed is the seam pass's (no predecessor in the tile)
#define FRT_TORN0 16u      // batch: the first / last frame runs past its shard's end (a terminal, no frame)
#define FRT_TORNZ 32u
#define FRT_OKZ 64u        // the last frame decoded (canonical layout)
#define FRT_PEB 128u       // peB holds P at the stream end (the stream's last tile)

// Batch: per shard, positions in the batch buffer.
struct ShardPos {
  unsigned long long first_fail;   // min (p << 8 | status), ~0
  unsigned long long first_meta;   // min p of a non-empty metadata frame, ~0
  unsigned long long term;         // min (q << 8 | class): where the shard's frames end before it does, ~0
  long long last_entry, last_state, lastop, lastp;   // max p, -1 (lastp: any frame)
  uint32_t bad, open;              // bad: replayed alone; open: a frame starts at the shard's first byte
  uint32_t rew, rmode;             // rew: entry indexes go back; rmode: this shard's ops claim slots (the rewind-mode pass over its tiles)
};

struct FrArgs {
  const uint8_t *buf;
  uint64_t B;
  uint32_t nunits, ntiles;
  const ulonglong2 *hmask;         // per unit: flagged pieces, of them those flagged in their last dword group
  const uint32_t *v, *g_slice, *g_shift;
  uint32_t *pl;                    // per unit: P at its start, relative to its tile's start
  uint32_t *ucb;                   // per unit: candidates of its tile before it
  FrTile *trec;
  uint32_t *tcnt;                  // per tile: its frames (FrTile.count, packed for the scans)
  ewal_entry *ents;
  uint64_t ecap;                   // single WAL: ents capacity
  uint64_t *mlist;                 // positions of metadata frames
  uint32_t mcap;
  uint64_t ri;                     // w.ri (single WAL)
  Small *ds;
  // rewind mode (single WAL, ReadAll's ents = append(ents[:Index-ri], e) with
  // indexes going back, wal/wal.go:173): every op claims its slot k with
  // atomicMax(own[k], 1 + position); a slot claimed twice is listed (clist)
  // and k_ents_fix stores the last op's entry there after the pass
  int rew;
  unsigned long long *own;
  uint32_t *clist;
  uint32_t ccap;
  // the tiles to run (nullptr: all ntiles): the rewind-mode pass over the
  // tiles of a batch's rewinding shards
  const uint32_t *tlist;
  uint32_t ntl;
  // without tlist: the tiles [t0, t0 + nrun) (nrun 0: all ntiles) -- a chunk
  // of the stream whose stream pass has completed (the overlapped pipeline)
  uint32_t t0, nrun;
  uint32_t *tick;                  // this launch's tile counter (zeroed before it)
  const uint32_t *vh;              // record-dense WALs: the first 128-B half's lin of every super-piece (k_stream), else null
  const uint32_t *ulin;            // EW_ULIN: every unit's lin (k_stream)
};
struct FrSeg {
  uint32_t ns;
  const uint64_t *soff;            // shard s = [soff[s], soff[s + 1])
  const uint64_t *ri;              // w.ri of every shard
  uint64_t *rbase;                 // ents region of every shard [ns + 1]
  ShardPos *sp;
  uint32_t *tcb;                   // candidates before every tile (k_tile_scan)
};

// the last shard s in [a, b) with soff[s] <= p
__device__ __forceinline__ uint32_t pos_shard_in(const uint64_t *__restrict__ soff, uint32_t a, uint32_t b, uint64_t p) {
  while (b - a > 1) {
    const uint32_t m = (a + b) >> 1;
    if (soff[m] <= p) a = m; else b = m;
  }
  return a;
}

// 64-bit lane shuffles
__device__ __forceinline__ uint64_t shfl64(uint64_t x, int l) {
  return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(x >> 32), l) << 32) | (uint32_t)__shfl((int)(uint32_t)x, l);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t x) {
  return ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(x >> 32), 1) << 32) | (uint32_t)__shfl_up((int)(uint32_t)x, 1);
}
__device__ __forceinline__ uint64_t shfl_down64(uint64_t x) {
  return ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(x >> 32), 1) << 32) |
         (uint32_t)__shfl_down((int)(uint32_t)x, 1);
}
__device__ __forceinline__ uint32_t rl32(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
  return ((uint64_t)rl32((uint32_t)(x >> 32), l) << 32) | rl32((uint32_t)x, l);
}

// the first lane whose (non-decreasing) inclusive count exceeds g
__device__ __forceinline__ int owner_lane(uint32_t incl, uint32_t g) {
  int lo = 0;
#pragma unroll
  for (int step = 32; step; step >>= 1) {
    const uint32_t x = (uint32_t)__shfl((int)incl, lo + step - 1);
    lo = x <= g ? lo + step : lo;
  }
  return lo;
}
// position of the k-th (0-based) set bit of m
__device__ __forceinline__ uint32_t nth_bit(unsigned long long m, uint32_t k) {
  const uint32_t c32 = (uint32_t)__popc((uint32_t)m);
  const bool hi = k >= c32;
  uint32_t w = hi ? (uint32_t)(m >> 32) : (uint32_t)m, base = hi ? 32u : 0u;
  k -= hi ? c32 : 0u;
#pragma unroll
  for (int s = 16; s; s >>= 1) {
    const uint32_t c = (uint32_t)__popc(w & ((1u << s) - 1u));
    const bool up = k >= c;
    k -= up ? c : 0u;
    w = up ? w >> s : w;
    base += up ? (uint32_t)s : 0u;
  }
  return base;
}

// Every exact frame-start candidate of a loaded piece as a bit mask (bit =
// byte offset in the piece): CAND_TEST's tests (wal_kernels.hip).
__device__ __forceinline__ unsigned long long cand_bits(const uint32_t (&D)[19], uint32_t fm, uint64_t off, uint64_t B) {
  unsigned long long m = 0;
#define CAND_ACTION m |= 1ull << (uint32_t)(p_ - off)
  if (fm & 0x80808080u) { CAND_TEST(0) CAND_TEST(1) CAND_TEST(2) CAND_TEST(3) }
  if (fm & 0x40404040u) { CAND_TEST(4) CAND_TEST(5) CAND_TEST(6) CAND_TEST(7) }
  if (fm & 0x20202020u) { CAND_TEST(8) CAND_TEST(9) CAND_TEST(10) CAND_TEST(11) }
  if (fm & 0x10101010u) { CAND_TEST(12) CAND_TEST(13) CAND_TEST(14) CAND_TEST(15) }
#undef CAND_ACTION
  return m;
}

// prefix_load_near with the unit's P given as a value (tile-local)
__device__ __forceinline__ void prefix_load_near_pw(uint64_t x, uint64_t B, uint32_t pw, const uint32_t *__restrict__ v,
                                                    const uint8_t *__restrict__ buf, PrefixNear &in) {
  const uint64_t w = x >> 12;
  const uint64_t x0 = x & ~(uint64_t)(EW_VPIECE - 1);
  const uint32_t k = (uint32_t)((x0 >> EW_VLOG) & (EW_VPU - 1));
  const uint32_t tail = (uint32_t)(x - x0);
  in.up = tail > EW_VPIECE / 2 && x0 + EW_VPIECE <= B;
  in.slow = tail > EW_VPIECE / 2 && !in.up;
  in.nk = k + in.up;
  in.lead = (uint32_t)(x & 15);
  const uint64_t base = in.up ? (x & ~15ull) : x0;
  in.n = in.up ? (uint32_t)(x0 + EW_VPIECE - base) : (in.slow ? 0u : tail);
  const uint4 *vq = (const uint4 *)(v + w * EW_VPU);
#pragma unroll
  for (int q = 0; q < EW_VPU / 4; ++q) in.vv[q] = (4u * q < in.nk) ? vq[q] : make_uint4(0, 0, 0, 0);
  const uint4 *dq = (const uint4 *)(buf + base);
#pragma unroll
  for (int q = 0; q < 8; ++q) in.dd[q] = (16u * q < in.n) ? dq[q] : make_uint4(0, 0, 0, 0);
  in.pw = pw;
}
// P(x) forward from its unit's start, pw = P there (rare paths)
__device__ __forceinline__ uint32_t prefix_at_pw(uint64_t x, uint32_t pw, const uint32_t *__restrict__ v,
                                                 const uint8_t *__restrict__ buf, const uint32_t *t4,
                                                 const uint32_t *svp) {
  PrefixIn in;
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
  in.pw = pw;
  return prefix_finish(in, t4, svp);
}

// p in the upper half of the stream's last, partial super-piece (no boundary
// after it): P forward from the unit start, and P(data start) moved by the
// same difference (canon_finish stepped the header from the unit's P)
__device__ __noinline__ void fr_decode_slow(const uint8_t *__restrict__ buf, uint64_t p, uint32_t pw,
                                            const uint32_t *__restrict__ v, const uint32_t *s_t16,
                                            const uint32_t *s_svp, const RecDesc &d, uint32_t &Pfo, uint32_t &Pfd) {
  const uint32_t P = prefix_at_pw(p, pw, v, buf, s_t16, s_svp);
  uint32_t delta = P ^ Pfo;
  for (uint64_t n = d.doff - p; n; --n) delta = s_t16[delta & 0xff] ^ (delta >> 8);   // S_1, byte by byte
  Pfd ^= delta;
  Pfo = P;
}

// P at the stream end B from its unit's start (pw, tile-local): the stream's
// last frame's P(data end), computed by the wave that ran the last tile
// through the LDS tables (the seam pass would step up to 255 bytes through
// global ones); out of line, once per call
__device__ __noinline__ uint32_t fr_prefix_end(const uint8_t *__restrict__ buf, uint64_t B, uint32_t pw,
                                               const uint32_t *__restrict__ v, const uint32_t *s_t16,
                                               const uint32_t *s_svp) {
  return prefix_at_pw(B, pw, v, buf, s_t16, s_svp);
}

// canon_finish (wal_kernels.hip) on the frame at p with P relative to the
// tile: pw = P at p's unit start.  VH: the prefix from the nearest 128-B
// boundary (vh[], prefix_load_near_vh), else the nearest 256-B one.
template <bool VH>
__device__ __forceinline__ bool fr_decode(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p, uint32_t pw,
                                          const uint32_t *__restrict__ v, const uint32_t *__restrict__ vh,
                                          const uint32_t *s_t16, const uint32_t *s_svp, const uint32_t *s_inv,
                                          const uint32_t *s_n128, uint32_t *w, RecDesc &d, int64_t &L, uint32_t &Pfo,
                                          uint32_t &Pfd) {
  CanonLoad<VH ? 2 : 1> ld;
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
  if constexpr (VH) prefix_load_near_vh(p, B, pw, v, vh, buf, ld.pin);
  else prefix_load_near_pw(p, B, pw, v, buf, ld.pin);
  const bool slow = ld.pin.slow;
  const bool ok = canon_finish<FR_THREADS, VH ? 2 : 1>(buf, B, p, nullptr, v, s_t16, s_svp, w, d, L, Pfo, Pfd, slow,
                                                       s_inv, ld, s_n128);
  if (slow) fr_decode_slow(buf, p, pw, v, s_t16, s_svp, d, Pfo, Pfd);
  return ok;
}

// candidates in unit u at positions < p (one whole wave: the exact tests
// again on the unit's flagged pieces)
__device__ uint32_t fr_incount(const uint8_t *__restrict__ buf, uint64_t B, const ulonglong2 *__restrict__ hmask,
                               uint64_t u, uint64_t p) {
  const int lane = threadIdx.x & 63;
  const ulonglong2 h = hmask[u];
  const uint64_t off = u * EW_WAVE_BYTES + (uint64_t)lane * EW_PIECE;
  uint32_t cnt = 0;
  if (((h.x >> lane) & 1ull) && off < p) {
    uint32_t D[19];
    if ((h.y >> lane) & 1ull) load_piece80(buf, B, off, D);
    else load_piece64(buf, B, off, D);
    const uint32_t fm = cand_filter(D);
    unsigned long long m = fm ? cand_bits(D, fm, off, B) : 0ull;
    const uint64_t lim = p - off;
    if (lim < 64) m &= (1ull << lim) - 1ull;
    cnt = (uint32_t)__popcll(m);
  }
  for (int o = 32; o; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o);
  return cnt;
}

// Candidates before stream position x (one whole wave): those of the tiles
// before x's tile (tcb when given, else summed here), of its units before
// x's unit (ucb) and of x's unit before x.
__device__ uint64_t fr_ordinal(const FrArgs &a, uint32_t tu, uint64_t x, const uint32_t *tcb) {
  const int lane = threadIdx.x & 63;
  const uint64_t u = x >> 12;
  if (u >= a.nunits) {
    unsigned long long s = 0;
    for (uint32_t t = (uint32_t)lane; t < a.ntiles; t += 64) s += a.tcnt[t];
    for (int o = 32; o; o >>= 1) s += (unsigned long long)__shfl_xor((long long)s, o);
    return s;
  }
  const uint32_t t = (uint32_t)(u / tu);
  unsigned long long before = 0;
  if (tcb) {
    before = tcb[t];
  } else {
    for (uint32_t i = (uint32_t)lane; i < t; i += 64) before += a.tcnt[i];
    for (int o = 32; o; o >>= 1) before += (unsigned long long)__shfl_xor((long long)before, o);
  }
  return before + a.ucb[u] + fr_incount(a.buf, a.B, a.hmask, u, x);
}

// decoder.decode's check + ReadAll's crc-record rule with P(data end) given
__device__ __forceinline__ int fr_check(const uint32_t *g_shift, int32_t type, uint32_t crc, uint32_t seed, uint32_t pfd,
                                        uint32_t pe, uint64_t dlen) {
  uint32_t chained;
  return fc_check_one(g_shift, type, crc, seed, pfd, pe, dlen, &chained);
}

// The carried frame (wave-uniform): the previous frame round's last frame,
// whose check waits for its successor.
struct FrCarry {
  uint64_t p, s, dlen;
  uint32_t crc, seed, pfd, sh;
  int32_t type;
  uint32_t flags;   // 1 valid, 2 decoded, 4 torn, 8 tile-first (its seed is the seam pass's), 16 has its seed
};

#ifdef FR_TIMING
// tools/ timing builds only: per wave, the cycles of each phase of k_frames
__device__ unsigned long long fr_tdbg[8192 * 8];
__device__ unsigned long long fr_sdbg[1024 * 4];   // k_frames_seam: per block, its loop and fr_result cycles
__device__ unsigned long long fr_sdbg2[1024 * 8];  // k_frames_seam thread 0: the loop's steps
__device__ unsigned long long fr_sdbg3[1024 * 8];  // k_frames_seam: per block, the max over its threads of each step
__device__ unsigned long long fr_rdbg[8];          // fr_result thread 0: clock at its steps
#define FR_RT(i) do { if (threadIdx.x == 0) fr_rdbg[i] = clock64(); } while (0)
__device__ unsigned long long fr_wt[8192 * 4];     // k_frames per wave: realtime at start, end; tiles run
#define FR_T(i) do { const unsigned long long t_ = clock64(); tacc[i] += t_ - tlast; tlast = t_; } while (0)
#else
#define FR_T(i) do {} while (0)
#define FR_RT(i) do {} while (0)
#endif

// The tile record's running fields (wave-uniform) and a batch's per-shard
// reductions folded over the rounds, kept in a per-wave LDS slot instead of
// registers: the frame loop is at the 168-VGPR / 104-SGPR limit of 12
// waves/CU, and these long-lived uniform values spilled (A/B: configs[0]
// post-stream -8 %, 128 shards -3 %; the carried frame and the piece rounds'
// per-lane results in LDS too: no gain / +11 %, profiles/r04/ab_notes.txt).
// FR_TR_LDS=0 keeps them in registers (A/B builds).
#ifndef FR_TR_LDS
#define FR_TR_LDS 1
#endif
struct FrTr {
  unsigned long long first_index, last_index, firstop_p, lastop_p;
  unsigned long long fail, last_entry1, last_state1, meta0;
  uint32_t nops, seam;
};
struct FrAcc {
  unsigned long long aff, afm;
  long long ale, als, alo, alp;
  uint32_t ash, pad;
};

template <bool SEG, int TSH, bool VH = false>
__global__ __launch_bounds__(FR_THREADS, 1) void k_frames(FrArgs a, FrSeg sg) {
#ifdef FR_TIMING
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = clock64();
#endif
  constexpr int TU = 1 << TSH;                       // units per tile
  constexpr int UPL = TSH >= 6 ? 1 << (TSH - 6) : 1; // units per lane
  constexpr int NL = TU / UPL;                       // lanes holding units (64, or TU < 64)
  constexpr int LB = 12 + (TSH >= 6 ? TSH - 6 : 0);  // log2 of a lane's span in bytes
  __shared__ uint32_t s_t16[16 * 256];               // slicing-by-16
  __shared__ uint32_t s_svp[1024];                   // S_256 byte tables
  __shared__ uint32_t s_nib[FR_NIB * 128];           // S_{2^0} .. S_{2^19}, nibble tables
#if EW_TAIL2
  __shared__ uint32_t s_inv[EW_TAIL_TABS * 128];     // the prefix tails' shifts by -128..128 (tail_shift)
#else
  __shared__ uint32_t s_inv[7 * 128];                // S_{2^0}^-1 .. S_{2^6}^-1
#endif
  __shared__ uint32_t s_win[20 * FR_THREADS];        // frame heads, transposed
  __shared__ uint32_t s_ucnt[FR_WAVES][TU];          // candidates per unit of each wave's tile
  __shared__ uint32_t s_pw[FR_WAVES][TU];            // P at every unit start of each wave's tile (tile-local)
#if FR_TR_LDS
  __shared__ FrTr s_tr[FR_WAVES];
  __shared__ FrAcc s_acc[FR_WAVES];
#endif
  Small *ds = a.ds;
  if (SEG && ds->fr_capfail) return;                 // ents regions past the capacity: the host grows them, reruns
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t wid = blockIdx.x * FR_WAVES + (uint32_t)wv, nwaves = gridDim.x * FR_WAVES;
  stage_lds<FR_THREADS>(s_t16, 16 * 256, [&](int i) { return a.g_slice[i]; });
  stage_lds<FR_THREADS>(s_svp, 1024, [&](int i) { return a.g_shift[EW_VLOG * 1024 + i]; });
  stage_lds<FR_THREADS>(s_nib, FR_NIB * 128, [&](int i) { return nib_src(a.g_shift, i); });
#if EW_TAIL2
  stage_lds<FR_THREADS>(s_inv, EW_TAIL_TABS * 128, [&](int i) { return a.g_shift[EW_TAIL_OFF + i]; });
#else
  stage_lds<FR_THREADS>(s_inv, 7 * 128, [&](int i) { return nib_src(a.g_shift + EW_SHIFT_LEVELS * 1024, i); });
#endif
  __syncthreads();   // the only barrier: every wave runs its own tiles from here on
  FR_T(0);
#ifdef FR_TIMING
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  uint32_t ntl_run = 0;
#endif
  uint32_t *ucnt = s_ucnt[wv];
  uint32_t *spw = s_pw[wv];
  uint32_t *w = s_win + tid;
  uint32_t rare = 0, irr = 0, rews = 0;   // rews: 1 rewind mode met an index rewind, 2 an entry below ri (no op)
  unsigned long long need_ecap = 0;
  const uint32_t nt_run = a.tlist ? a.ntl : (a.nrun ? a.nrun : a.ntiles);
  // every wave's first tile is its id; the rest are handed out by a counter
  // (tiles differ in work: a static stride leaves the waves uneven)
  uint32_t *tick = a.tick ? a.tick : &ds->fr_tick;
  auto next_tile = [&]() {
    uint32_t nx = 0;
    if (lane == 0) nx = nwaves + atomicAdd(tick, 1u);
    return rl32(nx, 0);
  };
  for (uint32_t ti = wid; ti < nt_run; ti = next_tile()) {
    const uint32_t t = a.tlist ? a.tlist[ti] : a.t0 + ti;
    const uint32_t u0 = t * TU;
#ifdef FR_TIMING
    ++ntl_run;
#endif
    const uint64_t ts = (uint64_t)u0 * EW_WAVE_BYTES;
    // ---- A: the tile's unit lins, P at every unit start (tile-local) ----
    uint32_t x[UPL];
    uint32_t pcs = 0, lcnt = 0;   // flagged pieces per unit of the lane (8 bits each), their sum
#if EW_ULIN
#pragma unroll
    for (int j = 0; j < UPL; ++j) {   // the unit lins k_stream stored
      const uint32_t u = u0 + UPL * lane + j;
      const bool in = u < a.nunits && (NL == 64 || lane < NL);
      const uint32_t c = in ? (uint32_t)__popcll(a.hmask[u].x) : 0u;
      pcs |= c << (8 * j);
      lcnt += c;
      x[j] = in ? a.ulin[u] : 0u;
    }
#else
    {
      uint4 vq[UPL][4];
#pragma unroll
      for (int j = 0; j < UPL; ++j) {
        const uint32_t u = u0 + UPL * lane + j;
        const bool in = u < a.nunits && (NL == 64 || lane < NL);
        const uint32_t c = in ? (uint32_t)__popcll(a.hmask[u].x) : 0u;
        pcs |= c << (8 * j);
        lcnt += c;
        const uint4 *vp = (const uint4 *)(a.v + (size_t)(in ? u : 0) * EW_VPU);
#pragma unroll
        for (int k = 0; k < 4; ++k) vq[j][k] = in ? vp[k] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < UPL; ++j) x[j] = vq[j][0].x;
#pragma unroll
      for (int k = 1; k < 16; ++k)
#pragma unroll
        for (int j = 0; j < UPL; ++j) {
          const uint4 &g = vq[j][k >> 2];
          const uint32_t d = (k & 3) == 0 ? g.x : (k & 3) == 1 ? g.y : (k & 3) == 2 ? g.z : g.w;
#if FR_HORNER_NIB
          x[j] = nib_apply(s_nib + EW_VLOG * 128, x[j]) ^ d;   // S_256, conflict-free nibble lookups
#else
          x[j] = tab_apply(s_svp, x[j]) ^ d;
#endif
        }
    }
#endif
#pragma unroll
    for (int j = 0; j < UPL; ++j)
      if (NL == 64 || lane < NL) ucnt[UPL * lane + j] = 0;
    uint32_t q = 0;
#pragma unroll
    for (int j = 0; j < UPL; ++j) q = nib_apply(s_nib + 12 * 128, q) ^ x[j];
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      const uint32_t o = (uint32_t)__shfl_up((int)q, 1 << d);
      if (lane >= (1 << d)) q = nib_apply(s_nib + (LB + d) * 128, o) ^ q;
    }
    const uint32_t agg = rl32(q, NL - 1);
    {
      uint32_t pwj = (uint32_t)__shfl_up((int)q, 1);
      if (lane == 0) pwj = 0;
#pragma unroll
      for (int j = 0; j < UPL; ++j) {
        if (j) pwj = nib_apply(s_nib + 12 * 128, pwj) ^ x[j - 1];
        const uint32_t u = u0 + UPL * lane + j;
        if (NL == 64 || lane < NL) {
          spw[UPL * lane + j] = pwj;
          if (u < a.nunits) fr_st32(a.pl + u, pwj);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    FR_T(1);
    // P at a unit start of this tile by its index in the tile
    auto pw_of = [&](uint32_t ul) { return spw[ul < (uint32_t)TU ? ul : 0u]; };
    // flagged pieces: per lane the count over its units, wave prefix
    const uint32_t lincl = wave_incl_sum(lcnt);
    const uint32_t Tf = rl32(lincl, 63);   // flagged pieces in the tile
    // batch: the tile's shard range
    uint32_t shlo = 0, shhi = 0;
    if (SEG) {
      shlo = pos_shard_in(sg.soff, 0, sg.ns, ts);
      shhi = pos_shard_in(sg.soff, shlo, sg.ns, ts + (uint64_t)TU * EW_WAVE_BYTES - 1);
    }
    // ---- B: a piece round -> per lane its piece's candidates (cm), piece offset, inclusive count ----
    auto piece_round = [&](uint32_t g0, unsigned long long &cm, uint64_t &poff, uint32_t &cinc) {
      const uint32_t gl = g0 + (uint32_t)lane;
      const bool live = gl < Tf;
      const uint32_t g = live ? gl : Tf - 1;
      const int ol = owner_lane(lincl, g);
      uint32_t r = g - ((uint32_t)__shfl((int)lincl, ol) - (uint32_t)__shfl((int)lcnt, ol));
      const uint32_t opcs = (uint32_t)__shfl((int)pcs, ol);
      uint32_t jsel = 0;
      bool found = false;
#pragma unroll
      for (int j = 0; j < UPL; ++j) {
        const uint32_t c = (opcs >> (8 * j)) & 0xff;
        const bool here = !found && r < c;
        jsel = here ? (uint32_t)j : jsel;
        r = (!found && !here) ? r - c : r;
        found = found || here;
      }
      const uint32_t ul = (uint32_t)ol * UPL + jsel;   // unit in the tile
      const ulonglong2 hm = a.hmask[min(u0 + ul, a.nunits - 1)];   // (an L2 hit: read in A)
      const unsigned long long mx = hm.x, m3 = hm.y;
      const uint32_t pc = nth_bit(mx, r);              // piece in the unit
      poff = ts + (uint64_t)ul * EW_WAVE_BYTES + (uint64_t)pc * EW_PIECE;
      cm = 0;
      if (live) {
        uint32_t D[19];
        if ((m3 >> pc) & 1ull) load_piece80(a.buf, a.B, poff, D);
        else load_piece64(a.buf, a.B, poff, D);
        const uint32_t fm = cand_filter(D);
        if (fm) cm = cand_bits(D, fm, poff, a.B);
      }
      const uint32_t c = (uint32_t)__popcll(cm);
      if (c) atomicAdd(&ucnt[ul], c);
      cinc = wave_incl_sum(c);
    };
    // ---- C: frame rounds ----
    FrCarry cy;
    cy.flags = 0;
    cy.p = cy.s = cy.dlen = 0;
    cy.crc = cy.seed = cy.pfd = cy.sh = 0;
    cy.type = 0;
    uint32_t nfr = 0;                 // frames of the tile so far
    bool ophas = false;               // the last op of the tile so far: its k and shard
    uint64_t opk = 0;
    uint32_t opsh = 0;
    // the tile's record (wave-uniform values; the first frame's fields are
    // stored where they are found)
#if FR_TR_LDS
    FrTr &tr = s_tr[wv];
#else
    FrTr tr;
#endif
    tr.nops = 0; tr.seam = 0; tr.first_index = tr.last_index = 0;
    tr.firstop_p = tr.lastop_p = 0;
    tr.fail = ~0ull; tr.last_entry1 = tr.last_state1 = 0; tr.meta0 = ~0ull;
    uint32_t tflags = 0;
    // batch: per-shard reductions folded while the rounds stay in one shard
#if FR_TR_LDS
    FrAcc &acc = s_acc[wv];
#else
    FrAcc acc;
#endif
    uint32_t &ash = acc.ash;
    unsigned long long &aff = acc.aff, &afm = acc.afm;
    long long &ale = acc.ale, &als = acc.als, &alo = acc.alo, &alp = acc.alp;
    ash = EW_NIL;
    aff = afm = ~0ull;
    ale = als = alo = alp = -1;
    auto aflush = [&]() {
      if (SEG && ash != EW_NIL && lane == 0) {
        ShardPos *A = sg.sp + ash;
        if (aff != ~0ull) atomicMin(&A->first_fail, aff);
        if (afm != ~0ull) atomicMin(&A->first_meta, afm);
        if (ale >= 0) atomicMax(&A->last_entry, ale);
        if (als >= 0) atomicMax(&A->last_state, als);
        if (alo >= 0) atomicMax(&A->lastop, alo);
        if (alp >= 0) atomicMax(&A->lastp, alp);
      }
      aff = afm = ~0ull;
      ale = als = alo = alp = -1;
    };
    // two piece rounds in registers: A (consumed from ca on) and B (the next one)
    unsigned long long cmA = 0, cmB = 0;
    uint64_t poA = 0, poB = 0;
    uint32_t ciA = 0, ciB = 0, TA = 0, TB = 0, ca = 0;
    uint32_t gnext = 0;
    bool haveB = false;
    if (Tf) {
      piece_round(0, cmA, poA, ciA);
      TA = rl32(ciA, 63);
      gnext = 64;
    }
    FR_T(2);
    bool first_round = true;
    for (;;) {
      while (!haveB && TA - ca < 63 && gnext < Tf) {   // keep 63 candidates ahead while pieces remain
        piece_round(gnext, cmB, poB, ciB);
        TB = rl32(ciB, 63);
        gnext += 64;
        haveB = true;
        if (TA == ca) {   // A spent: B becomes A
          cmA = cmB; poA = poB; ciA = ciB; TA = TB; ca = 0;
          haveB = false;
        }
      }
      FR_T(2);
      const uint32_t avail = (TA - ca) + (haveB ? TB : 0u);
      if (avail == 0) break;
      const uint32_t nnew = min(avail, 63u);
      const uint32_t last_lane = nnew;   // the round's last occupied lane: carried to the next round
      // lane i >= 1 takes the window's candidate i - 1
      const uint32_t fi = (uint32_t)lane - 1u;
      const bool isnew = lane >= 1 && fi < nnew;
      uint64_t p;
      {
        const uint32_t fa = ca + (isnew ? fi : 0u);
        const bool inA = fa < TA;
        const uint32_t fb = inA ? 0u : fa - TA;
        const int olA = owner_lane(ciA, inA ? fa : 0u);
        const int olB = owner_lane(ciB, fb);
        const unsigned long long mA = shfl64(cmA, olA), mB = shfl64(cmB, olB);
        const uint64_t pA = shfl64(poA, olA), pB = shfl64(poB, olB);
        const uint32_t eA = (uint32_t)__shfl((int)ciA, olA) - (uint32_t)__popcll(mA);
        const uint32_t eB = (uint32_t)__shfl((int)ciB, olB) - (uint32_t)__popcll(mB);
        p = inA ? pA + nth_bit(mA, fa - eA) : pB + nth_bit(mB, fb - eB);
      }
      const uint32_t ul = (uint32_t)((p >> 12) - u0);
      const uint32_t pwu = pw_of(ul);
      RecDesc d;
      int64_t L = 0;
      uint32_t Pfo = 0, Pfd = 0;
      bool ok = false;
      d.type = 0; d.crc = 0; d.dlen = 0; d.doff = p + 8; d.f0 = d.f1 = d.f2 = 0; d.edoff = 0; d.edlen = 0;
      d.enil = 1; d.etype = 0; d.dnil = 1;
      if (isnew) {
        ok = fr_decode<VH>(a.buf, a.B, p, pwu, a.v, a.vh, s_t16, s_svp, s_inv, s_nib + 7 * 128, w, d, L, Pfo, Pfd);
        if (!ok) { d.type = 0; d.dlen = 0; d.doff = p + 8; }
      }
      FR_T(3);
      uint64_t s = p + 8 + (uint64_t)L;
      uint32_t sh = 0;
      if (SEG && isnew) sh = shlo == shhi ? shlo : pos_shard_in(sg.soff, shlo, shhi + 1, p);
      // lane 0: the carried frame
      const bool cv = (cy.flags & 1u) != 0;
      if (lane == 0 && cv) {
        p = cy.p; s = cy.s; d.crc = cy.crc; d.type = cy.type; d.dlen = cy.dlen; d.doff = cy.s - cy.dlen;
        Pfd = cy.pfd; sh = cy.sh;
        ok = (cy.flags & 2u) != 0;
      }
      const bool occ = isnew || (lane == 0 && cv);
      const uint64_t S0 = SEG ? sg.soff[sh] : 0ull, E = SEG ? sg.soff[sh + 1] : a.B;
      const bool torn = SEG && occ && (lane == 0 ? (cy.flags & 4u) != 0 : s > E);
      const bool sfirst = occ && p == S0;   // the frame opens its shard (the WAL)
      // predecessor (lane - 1) and successor (lane + 1) in the round
      const uint32_t pcrc = (uint32_t)__shfl_up((int)d.crc, 1);
      const uint32_t psh = (uint32_t)__shfl_up((int)sh, 1);
      const bool pocc = __shfl_up((int)occ, 1) != 0;
      const uint64_t np = shfl_down64(p);
      const uint32_t npfo = (uint32_t)__shfl_down((int)Pfo, 1);
      const uint32_t nsh = (uint32_t)__shfl_down((int)sh, 1);
      const bool hasp = isnew && pocc;        // a predecessor in the tile
      // seed: a shard (WAL) starts from 0, else the predecessor's stored CRC
      bool hasseed;
      uint32_t seed;
      bool tfirst;
      if (lane == 0) {
        hasseed = (cy.flags & 16u) != 0;
        seed = cy.seed;
        tfirst = (cy.flags & 8u) != 0;
      } else {
        hasseed = sfirst || (hasp && (!SEG || psh == sh));
        seed = sfirst ? 0u : pcrc;
        tfirst = isnew && !hasp && !sfirst;
      }
      bool bad = false;    // batch: the frame takes its shard off the regular path
      if (isnew && !ok && !torn) {
        if (SEG) bad = true; else rare |= 1u;
      }
      if (SEG && isnew && !sfirst && hasp && psh != sh) bad = true;   // a shard opening elsewhere than its first byte
      if (SEG && isnew && sfirst) sg.sp[sh].open = 1u;
      if (SEG && isnew && torn) {   // a torn candidate: decoder.decode's terminal in its shard
        const uint64_t rem8 = E - p;
        int tst;
        if (rem8 < 8) tst = EWAL_ERR_UNEXPECTED_EOF;
        else {
          const uint64_t rem = rem8 - 8;
          tst = (uint64_t)L > rem ? (rem == 0 ? EWAL_OK : EWAL_ERR_UNEXPECTED_EOF) : -1;
        }
        if (tst < 0) bad = true;
        else atomicMin(&sg.sp[sh].term, (p << 8) | (uint32_t)tst);
      }
      // ---- checks of the occupied lanes whose successor is in the round ----
      const bool linked = occ && (uint32_t)lane < last_lane;
      if (linked) {
        if (!SEG) {
          if (np != s) irr = 1;
        } else if (nsh == sh) {
          if (np != s) bad = true;
        } else if (!torn && s != E) {   // the shard's last frame ends before the shard: the terminal at s
          const uint64_t rem8 = E - s;
          int tst;
          if (rem8 < 8) tst = EWAL_ERR_UNEXPECTED_EOF;
          else {
            const int64_t Lq = (int64_t)ld_le64_b(a.buf, a.B, s);
            const uint64_t rem = rem8 - 8;
            if (Lq < 0) tst = EWAL_PANIC_NEG_LENGTH;
            else if ((uint64_t)Lq > rem) tst = rem == 0 ? EWAL_OK : EWAL_ERR_UNEXPECTED_EOF;
            else tst = -1;   // a frame that fits but is no candidate: the general walk
          }
          if (tst < 0) bad = true;
          else atomicMin(&sg.sp[sh].term, (s << 8) | (uint32_t)tst);
        }
      }
      // P(data end): the successor's P at its start when the Data ends there
      // (canonical layout), else computed in this tile
      const uint64_t e = d.doff + d.dlen;
      const uint32_t ule = (uint32_t)((e >> 12) - u0);
      const uint32_t pwe = pw_of(ule);
      const bool chk = linked && !torn;
      uint32_t Pe = npfo;
      int st = 0;
      if (chk) {
        if (d.dlen && e != np) {
          if (ule < (uint32_t)TU) Pe = prefix_at_pw(e, pwe, a.v, a.buf, s_t16, s_svp);
          else if (SEG) bad = true;
          else rare |= 16u;
        }
        if (!tfirst && (!SEG || hasseed)) {
          if (d.type == 4) {
            if (seed != 0 && d.crc != seed) st = EWAL_ERR_WAL_CRC;
          } else {
            uint32_t computed = seed;
            if (d.dlen && !(EW_FR_ABL & 4)) {
              uint32_t xs = seed ^ 0xffffffffu ^ Pfd;
              uint64_t m = d.dlen;
              int lvl = 0;
#if FR_DLEN2
              // the low 12 bits in three rounds through the tail tables (S_b,
              // S_{16a}: tables 0..8 and 50..56, S_{256a}: 57..71), the rest
              // bit by bit
              {
                const uint32_t lo4 = (uint32_t)m & 15u, a4 = (uint32_t)(m >> 4) & 15u, h4 = (uint32_t)(m >> 8) & 15u;
                xs = nib_apply(s_inv + (9u + lo4) * 128, xs);
                xs = nib_apply(s_inv + (a4 <= 8u ? a4 : 41u + a4) * 128, xs);
                xs = nib_apply(s_inv + (h4 ? 56u + h4 : 0u) * 128, xs);
                m >>= 12;
                lvl = 12;
              }
#endif
              for (; m; ++lvl, m >>= 1)
                if (m & 1) xs = lvl < FR_NIB ? nib_apply(s_nib + lvl * 128, xs) : gshift_pow2(a.g_shift, lvl, xs);
              computed = xs ^ Pe ^ 0xffffffffu;
            }
            // a range of a WAL split inside a file: frame 0's check is the caller's
            const bool defer0 = !SEG && p == 0 && ds->defer_first;
            if (computed != d.crc && !defer0) st = EWAL_ERR_RECORD_CRC;
            else if (d.type != 1 && d.type != 2 && d.type != 3) st = EWAL_ERR_UNEXPECTED_TYPE;
          }
        }
      }
      FR_T(4);
      // the tile's first frame: its operands for the seam pass, stored by the
      // lane holding it (lane 1 of the first round; its P(data end) by the
      // lane that checks it)
      if (first_round) {
        if (lane == 1) {
          FrTile *T = a.trec + t;
          T->p0 = p;
          T->pfo0 = Pfo;
          T->type0 = (int32_t)(d.type < 0 || d.type > 1000 ? 1000 : d.type);
          T->crc0 = d.crc;
          T->pfd0 = Pfd;
          T->dlen0 = d.dlen;
          if (last_lane > 1) T->pe0 = Pe;
        }
        tflags |= (rl32((uint32_t)tfirst, 1) ? FRT_T0 : 0u) | (rl32((uint32_t)torn, 1) ? FRT_TORN0 : 0u) |
                  (last_lane > 1 ? FRT_PE0 : 0u);
      } else if ((cy.flags & 8u) && cv) {   // the carried frame is the tile's first: its successor is here
        if (lane == 0) a.trec[t].pe0 = Pe;
        tflags |= FRT_PE0;
      }
      // ---- per new frame: ReadAll's rules, entry ops ----
      uint64_t ri = a.ri;
      if (SEG) ri = sg.ri[sh];
      const bool ent = isnew && ok && !torn && d.type == 2;
      const bool op = ent && d.f1 >= ri;
      if (!SEG && ent && !op) rews |= 2u;   // an entry below ri: the range info's descriptors decide (ewal_copy_range_info)
      const unsigned long long mo = __ballot(op);
      const unsigned long long below = mo & ((1ull << lane) - 1ull);
      const int pol = below ? 63 - __clzll((long long)below) : lane;
      const uint64_t kp_l = (uint64_t)__shfl((long long)(d.f1 - ri), pol);
      const uint32_t shp_l = (uint32_t)__shfl((int)sh, pol);
      if (op) {
        const uint64_t k = d.f1 - ri;
        bool has = false;
        uint64_t kq = 0;
        if (below) {
          if (!SEG || shp_l == sh) { has = true; kq = kp_l; }
        } else if (ophas && (!SEG || opsh == sh)) {
          has = true;
          kq = opk;
        }
        // without an earlier op in the tile: none at all when the shard
        // opened in this tile, else the seam pass applies the rule
        const bool seam_op = !has && !below && !ophas && !(SEG && S0 >= ts);
        if (!seam_op) {
          bool gap;
          if (has) {
            // an index rewind: the rewind-mode pass (single WAL), the shard replayed alone (batch)
            if (k <= kq) {
              if (SEG) sg.sp[sh].rew = (a.rew && sg.sp[sh].rmode) ? 2u : 1u;   // 2: its claims are in this pass
              else if (!a.rew) rare |= 2u;
              else rews |= 1u;
            }
            gap = k > kq && k - kq > 1;
          } else {
            gap = k > 0;
          }
          if (gap) st = st ? st : EWAL_PANIC_INDEX_GAP;
        }
        if (SEG) {   // op k of the shard: its region's entry k
          const uint64_t rb = sg.rbase[sh], room = sg.rbase[sh + 1] - rb;
          if (k < room) {
            if (EW_ENTS_SC1) store_entry_sc1(a.ents + rb + k, ewal_entry{d.f0, d.f1, d.edoff - S0, d.edlen, d.etype, (int32_t)d.enil});
            else a.ents[rb + k] = ewal_entry{d.f0, d.f1, d.edoff - S0, d.edlen, d.etype, (int32_t)d.enil};
            if (a.rew && sg.sp[sh].rmode && atomicMax(&a.own[rb + k], (unsigned long long)(p + 1))) {   // a slot written twice
              const uint32_t ci = atomicAdd(&ds->fr_ncl, 1u);
              if (ci < a.ccap) a.clist[ci] = (uint32_t)(rb + k); else rare |= 64u;
            }
          }
        } else if (k < a.ecap) {
          if (EW_ENTS_SC1 >= 2) store_entry_sc1(a.ents + k, ewal_entry{d.f0, d.f1, d.edoff, d.edlen, d.etype, (int32_t)d.enil});
          else store_entry_nt(a.ents + k, ewal_entry{d.f0, d.f1, d.edoff, d.edlen, d.etype, (int32_t)d.enil});
          if (a.rew && atomicMax(&a.own[k], (unsigned long long)(p + 1))) {   // a slot written twice
            const uint32_t ci = atomicAdd(&ds->fr_ncl, 1u);
            if (ci < a.ccap) a.clist[ci] = (uint32_t)k; else rare |= 64u;
          }
        } else {
          rare |= 4u;
          need_ecap = max(need_ecap, (unsigned long long)(k + 1));
        }
      }
      if (mo) {
        const int wf = __ffsll((long long)mo) - 1, wl = 63 - __clzll((long long)mo);
        if (!ophas) {
          tr.first_index = rl64(d.f1, wf);
          tr.firstop_p = rl64(p, wf);
          const uint32_t shf = rl32(sh, wf);
          tr.seam = !(SEG && sg.soff[shf] >= ts);
        }
        tr.last_index = rl64(d.f1, wl);
        tr.lastop_p = rl64(p, wl);
        tr.nops += (uint32_t)__popcll(mo);
        ophas = true;
        opk = rl64(d.f1 - ri, wl);
        opsh = rl32(sh, wl);
      }
      // metadata frames: ReadAll's metadata rule runs after the pass
      if (isnew && ok && !torn && d.type == 1) {
        const uint32_t mi = atomicAdd(&ds->nmeta, 1u);
        if (mi < a.mcap) a.mlist[mi] = p; else rare |= 8u;
      }
      FR_T(5);
      // reductions over the round (lanes are in stream order)
      const bool rlive = isnew && !torn;
      const unsigned long long mf = __ballot(occ && st != 0), me = __ballot(rlive && d.type == 2),
                               ms = __ballot(rlive && d.type == 3), mm = __ballot(rlive && d.type == 1 && d.dlen > 0),
                               ma = __ballot(rlive);
      if (SEG) {
        const int l0 = __ffsll((long long)__ballot(occ)) - 1;
        const uint32_t sh0 = rl32(sh, l0);
        if (__ballot(occ && sh != sh0) == 0ull) {   // the round in one shard: folded
          if (ash != sh0) { aflush(); ash = sh0; }
          if (mf) {
            const int fl = __ffsll((long long)mf) - 1;
            aff = min(aff, (unsigned long long)(rl64(p, fl) << 8) | rl32((uint32_t)st, fl));
          }
          if (me) ale = max(ale, (long long)rl64(p, 63 - __clzll((long long)me)));
          if (ms) als = max(als, (long long)rl64(p, 63 - __clzll((long long)ms)));
          if (mm) afm = min(afm, (unsigned long long)rl64(p, __ffsll((long long)mm) - 1));
          if (ma) alp = max(alp, (long long)rl64(p, 63 - __clzll((long long)ma)));
          if (mo) alo = max(alo, (long long)rl64(p, 63 - __clzll((long long)mo)));
        } else {                                     // a shard boundary in the round: lane by lane
          ShardPos *A = sg.sp + sh;
          if (occ && st != 0) atomicMin(&A->first_fail, (p << 8) | (uint32_t)st);
          if (rlive && d.type == 2) atomicMax(&A->last_entry, (long long)p);
          if (rlive && d.type == 3) atomicMax(&A->last_state, (long long)p);
          if (rlive && d.type == 1 && d.dlen > 0) atomicMin(&A->first_meta, (unsigned long long)p);
          if (op) atomicMax(&A->lastop, (long long)p);
          if (rlive) atomicMax(&A->lastp, (long long)p);
        }
        if (bad) atomicOr(&sg.sp[sh].bad, 1u);
      } else {
        if (mf) {
          const int fl = __ffsll((long long)mf) - 1;
          tr.fail = min(tr.fail, (unsigned long long)(rl64(p, fl) << 8) | rl32((uint32_t)st, fl));
        }
        if (me) tr.last_entry1 = max(tr.last_entry1, rl64(p, 63 - __clzll((long long)me)) + 1);
        if (ms) tr.last_state1 = max(tr.last_state1, rl64(p, 63 - __clzll((long long)ms)) + 1);
        if (mm) tr.meta0 = min(tr.meta0, rl64(p, __ffsll((long long)mm) - 1));
      }
      // the round's last frame waits for its successor: carried
      {
        const int cl = (int)last_lane;
        FrCarry n;
        n.p = rl64(p, cl);
        n.s = rl64(s, cl);
        n.dlen = rl64(d.dlen, cl);
        n.crc = rl32(d.crc, cl);
        n.seed = rl32(seed, cl);
        n.pfd = rl32(Pfd, cl);
        n.sh = rl32(sh, cl);
        n.type = (int32_t)rl32((uint32_t)(int32_t)(d.type < 0 || d.type > 1000 ? 1000 : d.type), cl);
        n.flags = 1u | (rl32((uint32_t)ok, cl) ? 2u : 0u) | (rl32((uint32_t)torn, cl) ? 4u : 0u) |
                  (rl32((uint32_t)tfirst, cl) ? 8u : 0u) | (rl32((uint32_t)hasseed, cl) ? 16u : 0u);
        cy = n;
      }
      first_round = false;
      nfr += nnew;
      if (ca + nnew <= TA) {
        ca += nnew;
      } else {
        const uint32_t fromB = ca + nnew - TA;
        cmA = cmB; poA = poB; ciA = ciB; TA = TB; ca = fromB;
        haveB = false;
      }
      if (ca == TA && haveB) {
        cmA = cmB; poA = poB; ciA = ciB; TA = TB; ca = 0;
        haveB = false;
      }
      FR_T(6);
    }
    if (SEG) aflush();
    // per unit: the tile's candidates before it
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    {
      uint32_t c[UPL], cs = 0;
#pragma unroll
      for (int j = 0; j < UPL; ++j) {
        c[j] = (NL == 64 || lane < NL) ? ucnt[UPL * lane + j] : 0u;
        cs += c[j];
      }
      const uint32_t inc = wave_incl_sum(cs);
      uint32_t run = inc - cs;
#pragma unroll
      for (int j = 0; j < UPL; ++j) {
        const uint32_t u = u0 + UPL * lane + j;
        if (u < a.nunits && (NL == 64 || lane < NL)) fr_st32(a.ucb + u, run);
        run += c[j];
      }
    }
    if (lane == 0) {
      FrTile *T = a.trec + t;
      T->count = nfr;
      a.tcnt[t] = nfr;
      T->agg = agg;
      if (nfr) {   // the last frame: the carried one
        T->pz = cy.p;
        T->sz = cy.s;
        T->crcz = cy.crc;
        T->typez = cy.type;
        T->seedz = cy.seed;
        T->pfdz = cy.pfd;
        T->dlenz = cy.dlen;
        T->flags = tflags | (((cy.flags & 16u) && !(cy.flags & 8u)) ? FRT_SEEDZ : 0u) |
                   ((cy.flags & 4u) ? FRT_TORNZ : 0u) | ((cy.flags & 2u) ? FRT_OKZ : 0u);
        T->nops = tr.nops;
        T->seam = tr.seam;
        T->first_index = tr.first_index;
        T->last_index = tr.last_index;
        T->firstop_p = tr.firstop_p;
        T->lastop_p = tr.lastop_p;
        T->fail = tr.fail;
        T->last_entry1 = tr.last_entry1;
        T->last_state1 = tr.last_state1;
        T->meta0 = tr.meta0;
        atomicAdd(&ds->total, (unsigned long long)nfr);
        if ((uint64_t)u0 + TU >= a.nunits) {   // the stream's (the batch's) last tile
          T->peB = fr_prefix_end(a.buf, a.B, spw[(uint32_t)((a.B >> 12) - u0)], a.v, s_t16, s_svp);
          T->flags |= FRT_PEB;
        }
      }
    }
    FR_T(7);
  }
#ifdef FR_TIMING
  if (lane == 0 && wid < 8192) {
    for (int i = 0; i < 8; ++i) fr_tdbg[wid * 8 + i] = tacc[i];
    fr_wt[wid * 4] = rt0;
    fr_wt[wid * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    fr_wt[wid * 4 + 2] = ntl_run;
  }
#endif
  uint32_t rr = rare;
  for (int o = 32; o; o >>= 1) rr |= (uint32_t)__shfl_xor((int)rr, o);
  if (lane == 0 && rr) atomicOr(&ds->fc.rare, rr);
  if (__ballot(irr) && lane == 0) atomicOr(&ds->irregular, 1u);
  if (!SEG) {
    uint32_t rw = rews;
    for (int o = 32; o; o >>= 1) rw |= (uint32_t)__shfl_xor((int)rw, o);
    if (lane == 0 && (rw & 1u)) atomicOr(&ds->fr_rews, 1u);
    if (lane == 0 && (rw & 2u)) atomicOr(&ds->fr_below, 1u);
  }
  for (int o = 32; o; o >>= 1)
    need_ecap = max(need_ecap, (unsigned long long)__shfl_xor((long long)need_ecap, o));
  if (lane == 0 && need_ecap) atomicMax(&ds->fr_need, need_ecap);
}

// ---- seam pass --------------------------------------------------------------
// decoder.decode's check + ReadAll's crc-record rule, P(data end) given;
// defer: frame 0 of a range split inside a file (its CRC check is the caller's)
// S_n from the seam pass's LDS nibble tables (S_{2^0} .. S_{2^23}), the
// global byte tables above them
#define SEAM_NIB 24
#ifndef SEAM_DIG
#define SEAM_DIG 1   // the seam pass's shifts by hex digits (<= 5 table rounds below 2^20) instead of bit by bit
#endif
// S_n(x): s_n holds S_{2^m} (m < SEAM_NIB), then (SEAM_DIG) the digit tables
// S_{d 16^p} (crc_math.h EW_DIG_*), one round per nonzero hex digit below 2^20
#define SEAM_LDS (SEAM_NIB * 128 + (SEAM_DIG ? EW_DIG_TABS * 128 : 0))
__device__ __forceinline__ uint32_t seam_shift(const uint32_t *s_n, const uint32_t *g_shift, uint64_t n, uint32_t x) {
  const uint32_t *s_dg = s_n + SEAM_NIB * 128;   // (the kernels' s_n arrays: SEAM_LDS words)
  int m = 0;
  if (SEAM_DIG) {
    for (int p = 0; p < EW_DIG_POS && n; ++p, n >>= 4) {
      const uint32_t d = (uint32_t)n & 15u;
      if (d) x = nib_apply(s_dg + (p * 15 + d - 1) * 128, x);
    }
    m = 4 * EW_DIG_POS;
  }
  for (; n; ++m, n >>= 1)
    if (n & 1) x = m < SEAM_NIB ? nib_apply(s_n + m * 128, x) : gshift_pow2(g_shift, m, x);
  return x;
}
__device__ __forceinline__ int fr_check(const uint32_t *s_n, const uint32_t *g_shift, int32_t type, uint32_t crc,
                                        uint32_t seed, uint32_t pfd, uint32_t pe, uint64_t dlen, bool defer) {
  if (type == 4) return (seed != 0 && crc != seed) ? EWAL_ERR_WAL_CRC : 0;
  uint32_t computed = seed;
  if (dlen) computed = seam_shift(s_n, g_shift, dlen, seed ^ 0xffffffffu ^ pfd) ^ pe ^ 0xffffffffu;
  if (computed != crc && !defer) return EWAL_ERR_RECORD_CRC;
  return (type != 1 && type != 2 && type != 3) ? EWAL_ERR_UNEXPECTED_TYPE : 0;
}

// lin[ts_a, ts_b): the aggregates of tiles a .. b-1 (Horner, S_{tile bytes})
__device__ uint32_t fr_span_lin(const FrTile *__restrict__ trec, uint32_t a, uint32_t b, const uint32_t *s_n,
                                int tlog) {
  uint32_t acc = 0;
  for (uint32_t i = a; i < b; ++i) acc = nib_apply(s_n + tlog * 128, acc) ^ trec[i].agg;
  return acc;
}
// P(e) in tile ta's reference for a record of tile ta whose Data ends at e
// (ts_ta <= e <= B): S_{e - ts_b}(lin[ts_ta, ts_b)) ^ Pl_b(e), b = e's tile
__device__ uint32_t fr_pe_far(const FrArgs &a, const uint32_t *s_n, uint32_t ta, uint64_t e, uint32_t tu, int tlog) {
  uint64_t ue = e >> 12;
  if (ue >= a.nunits) ue = a.nunits - 1;
  const uint32_t tb = (uint32_t)(ue / tu);
  const uint64_t tsb = (uint64_t)tb * tu * EW_WAVE_BYTES;
  const uint32_t ple = prefix_at_pw(e, a.pl[ue], a.v, a.buf, a.g_slice, a.g_shift + EW_VLOG * 1024);
  if (tb <= ta) return ple;
  return seam_shift(s_n, a.g_shift, e - tsb, fr_span_lin(a.trec, ta, tb, s_n, tlog)) ^ ple;
}

// decoder.decode's terminal at q (no frame starts there) in a shard ending at
// E: its class, or -1 when a frame fits there (the general walk decides)
__device__ __forceinline__ int fr_terminal(const uint8_t *buf, uint64_t B, uint64_t q, uint64_t E) {
  if (E - q < 8) return EWAL_ERR_UNEXPECTED_EOF;
  const int64_t Lq = (int64_t)ld_le64_b(buf, B, q);
  const uint64_t rem = E - q - 8;
  if (Lq < 0) return EWAL_PANIC_NEG_LENGTH;
  if ((uint64_t)Lq > rem) return rem == 0 ? EWAL_OK : EWAL_ERR_UNEXPECTED_EOF;
  return -1;
}

// The single WAL's result after the seam pass (its last workgroup):
// ReadAll's metadata rule over the listed metadata frames, the frames the
// result names re-read from the stream, the failing frame's ordinal.
template <int TSH>
__device__ void fr_result(const FrArgs &a, ResultDev *o, Small *h, uint4 (*s_w)[6], RecDesc *s_d,
                          unsigned long long *s_ord, ResultDev *s_res) {
  Small *ds = a.ds;
  const uint32_t tid = threadIdx.x;
  const uint64_t K = ds->total;
  const bool valid = K && K < 0xffffff00ull && !ds->irregular && !ds->fc.rare && ds->pos0 == 0 && !ds->errflag;
  if (!valid) {
    __syncthreads();
    if (tid == 0) {
      ds->spec_n = 0;
      *h = *ds;
    }
    return;
  }
  FR_RT(0);
  const uint64_t fm = ds->fc.meta_inv ? ~ds->fc.meta_inv : ~0ull;
  if (fm != ~0ull && ds->nmeta > 1) {
    const RecDesc m = fc_frame_fields(a.buf, a.B, fm, s_w[tid]);
    for (uint32_t i = tid; i < ds->nmeta; i += blockDim.x) {
      const uint64_t p = a.mlist[i];
      if (p <= fm) continue;
      const RecDesc d = fc_frame_fields(a.buf, a.B, p, s_w[tid]);
      bool eq = d.dlen == m.dlen;
      for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = a.buf[d.doff + k] == a.buf[m.doff + k];
      if (!eq) atomicMax(&ds->fc.fail_inv, ~((p << 8) | EWAL_ERR_METADATA_CONFLICT));
    }
  }
  FR_RT(1);
  if (tid == 0) *s_ord = 0;
  __threadfence();
  __syncthreads();
  FR_RT(2);
  const unsigned long long key = ds->fc.fail_inv ? ~ds->fc.fail_inv : ~0ull;
  const uint64_t le = ds->fr.le, ls = ds->fr.ls, lo = ds->fr.lo;
  const long long want[5] = {key != ~0ull ? (long long)(key >> 8) : -1, le ? (long long)(le - 1) : -1,
                             ls ? (long long)(ls - 1) : -1, fm != ~0ull ? (long long)fm : -1,
                             lo ? (long long)(lo - 1) : -1};
  // the frames the result names (wave 1) while the failing frame's ordinal is summed
  if (tid >= 64 && tid < 69 && want[tid - 64] >= 0)
    s_d[tid - 64] = fc_frame_fields(a.buf, a.B, (uint64_t)want[tid - 64], s_w[tid]);
  if (key != ~0ull) {   // the failing frame's ordinal: the tiles before it summed by the whole workgroup
    const uint64_t x = key >> 8, u = x >> 12;
    const uint32_t tx = u < a.nunits ? (uint32_t)(u >> TSH) : a.ntiles;
    unsigned long long part = 0;
#pragma unroll 8
    for (uint32_t i = tid; i < tx; i += blockDim.x) part += a.tcnt[i];
    for (int o = 32; o; o >>= 1) part += (unsigned long long)__shfl_xor((long long)part, o);
    if ((tid & 63) == 0 && part) atomicAdd(s_ord, part);
    if (u < a.nunits && tid < 64) {   // the tile's units before x's, and x's unit before x
      const unsigned long long in = a.ucb[u] + fr_incount(a.buf, a.B, a.hmask, u, x);
      if (tid == 0) atomicAdd(s_ord, in);
    }
  }
  __syncthreads();
  FR_RT(3);
  // the result composed in LDS by thread 0, then written to host-mapped
  // memory by a whole wave (wide PCIe writes instead of one lane's stores)
  ResultDev &res = *s_res;
#if FR_COMPOSE_W
  // (the zeroing and the named frames' copies by the first wave, dword-wise;
  // thread 0 then sets the scalar fields -- one wave's LDS ops stay in order)
  if (tid < 64) {
    static_assert(sizeof(RecDesc) % 4 == 0 && sizeof(RecDesc) / 4 <= 64, "a frame's copy in one wave step");
    uint32_t *rw = (uint32_t *)&res;
    for (uint32_t i = tid; i < sizeof(ResultDev) / 4; i += 64) rw[i] = 0u;
    constexpr uint32_t NW = sizeof(RecDesc) / 4;
    if (tid < NW) {
      const uint32_t *sw = (const uint32_t *)s_d;
      if (key != ~0ull) rw[offsetof(ResultDev, fail) / 4 + tid] = sw[0 * NW + tid];
      if (le) rw[offsetof(ResultDev, lastent) / 4 + tid] = sw[1 * NW + tid];
      if (ls) rw[offsetof(ResultDev, sd) / 4 + tid] = sw[2 * NW + tid];
      if (fm != ~0ull) rw[offsetof(ResultDev, md) / 4 + tid] = sw[3 * NW + tid];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // (the dword stores before thread 0's fields)
    __builtin_amdgcn_wave_barrier();
  }
  if (tid == 0) {
    res.agg.first_fail = key != ~0ull ? *s_ord : ~0ull;
    res.agg.last_entry = le ? 0 : -1;
    res.agg.last_state = ls ? 0 : -1;
    res.agg.first_meta = fm != ~0ull ? 0ull : ~0ull;
    if (key != ~0ull) res.fail.st = (int32_t)(key & 0xff);
    res.last.chained = ds->fc.last_chained;
    res.nops = (uint32_t)ds->fr.nops;
    res.klast = lo ? s_d[4].f1 - a.ri : 0;
    res.errflag = ds->errflag;
    ds->spec_n = (uint32_t)K;
  }
#else
  if (tid == 0) {
    memset(&res, 0, sizeof(res));
    res.agg.first_fail = key != ~0ull ? *s_ord : ~0ull;
    res.agg.last_entry = le ? 0 : -1;
    res.agg.last_state = ls ? 0 : -1;
    res.agg.first_meta = fm != ~0ull ? 0ull : ~0ull;
    if (key != ~0ull) {
      res.fail = s_d[0];
      res.fail.st = (int32_t)(key & 0xff);
    }
    if (le) res.lastent = s_d[1];
    if (ls) res.sd = s_d[2];
    if (fm != ~0ull) res.md = s_d[3];
    res.last.chained = ds->fc.last_chained;
    res.nops = (uint32_t)ds->fr.nops;
    res.klast = lo ? s_d[4].f1 - a.ri : 0;
    res.errflag = ds->errflag;
    ds->spec_n = (uint32_t)K;
  }
#endif
  __threadfence_block();
  __syncthreads();
  FR_RT(4);
  if (tid < 64) {
    static_assert(sizeof(ResultDev) % 4 == 0 && sizeof(Small) % 4 == 0, "dword copies");
    const uint32_t *rs = (const uint32_t *)&res;
    uint32_t *rd = (uint32_t *)o;
    for (uint32_t i = tid; i < sizeof(ResultDev) / 4; i += 64) rd[i] = rs[i];
    const uint32_t *ss = (const uint32_t *)ds;
    uint32_t *sd = (uint32_t *)h;
    for (uint32_t i = tid; i < sizeof(Small) / 4; i += 64) sd[i] = ss[i];
  }
  FR_RT(5);
}

// One thread per tile: the checks of the tile's first frame (its seed from
// the previous tile with frames) and last frame (its P(data end) from the
// next), the links between them, the gap rule of the tile's first entry op;
// single WAL: the fold of the tiles' reductions and, in the last workgroup,
// the result.
template <bool SEG, int TSH>
__global__ __launch_bounds__(256) void k_frames_seam(FrArgs a, FrSeg sg, ResultDev *o, Small *h) {
  constexpr uint32_t TU = 1u << TSH;
  constexpr int TLOG = 12 + TSH;
  constexpr uint64_t TB = (uint64_t)TU * EW_WAVE_BYTES;
  __shared__ unsigned long long s_red[6];   // fail, meta, le, ls, lo, nops
  __shared__ uint32_t s_last;
  __shared__ uint4 s_w[SEG ? 1 : 256][6];
  __shared__ RecDesc s_d[SEG ? 1 : 6];
  __shared__ unsigned long long s_ord;
  __shared__ ResultDev s_res[SEG ? 1 : 1];
  __shared__ uint32_t s_n[SEAM_LDS];  // S_{2^m} nibble tables, m < 24, then the digit tables
  static_assert(TLOG < SEAM_NIB, "tile shifts from the LDS tables");
  Small *ds = a.ds;
  if (SEG && ds->fr_capfail) return;
#ifdef FR_TIMING
  const unsigned long long t_seam0 = clock64();
#endif
  stage_lds<256>(s_n, SEAM_NIB * 128, [&](int i) { return nib_src(a.g_shift, i); });
  if (SEAM_DIG) stage_lds<256>(s_n + SEAM_NIB * 128, EW_DIG_TABS * 128, [&](int i) { return a.g_shift[EW_DIG_OFF + i]; });
  if (!SEG && threadIdx.x == 0) {
    s_red[0] = s_red[1] = ~0ull;
    s_red[2] = s_red[3] = s_red[4] = s_red[5] = 0;
  }
  __syncthreads();
#ifdef FR_TIMING
  unsigned long long tq[8] = {(unsigned long long)clock64(), 0, 0, 0, 0, 0, 0, 0};
#define SEAM_T(i) do { if (!tq[i]) tq[i] = clock64(); } while (0)
#else
#define SEAM_T(i) do {} while (0)
#endif
  unsigned long long fail = ~0ull, meta = ~0ull, le = 0, ls = 0, lo = 0, nops = 0;
  auto badsh = [&](uint32_t s) { atomicOr(&sg.sp[s].bad, 1u); };
  auto key_at = [&](uint32_t s, uint64_t p, int st) {
    const unsigned long long k = (p << 8) | (uint32_t)st;
    if (SEG) atomicMin(&sg.sp[s].first_fail, k);
    else fail = min(fail, k);
  };
  const uint32_t nt_run = a.tlist ? a.ntl : a.ntiles;
  for (uint32_t ti = blockIdx.x * blockDim.x + threadIdx.x; ti < nt_run; ti += gridDim.x * blockDim.x) {
    const uint32_t t = a.tlist ? a.tlist[ti] : ti;
    const FrTile T = a.trec[t];
    // the neighbours' fields loaded together with T: the usual case (both
    // hold frames, the previous one ops) needs no further round trip
    const bool hp = t > 0, hn = t + 1 < a.ntiles;
    const uint32_t cp = hp ? a.tcnt[t - 1] : 0u, cn = hn ? a.tcnt[t + 1] : 0u;
    const FrTile *TP = a.trec + (hp ? t - 1 : t), *TN = a.trec + (hn ? t + 1 : t);
    const uint64_t P_pz = TP->pz, P_sz = TP->sz, P_lastop = TP->lastop_p, P_lastidx = TP->last_index;
    const uint32_t P_crcz = TP->crcz, P_nops = TP->nops;
    const uint64_t N_p0 = TN->p0;
    const uint32_t N_pfo0 = TN->pfo0, T_agg = T.agg;
    if (!T.count) continue;
#ifdef FR_TIMING
    if (threadIdx.x == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    SEAM_T(1);
    // ---- the previous frame: the last of the nearest earlier tile with frames ----
    int64_t pv = (int64_t)t - 1;
    uint32_t sc = 0;
    bool far = false;
    if (!(hp && cp)) {
      while (pv >= 0 && a.tcnt[pv] == 0) {
        if (++sc > FR_SCAN) { far = true; break; }
        --pv;
      }
    }
    const uint32_t sh0 = SEG ? pos_shard_in(sg.soff, 0, sg.ns, T.p0) : 0u;
    const bool sfirst0 = T.p0 == (SEG ? sg.soff[sh0] : 0ull);
    uint32_t seed0 = 0;
    bool seeded0 = sfirst0;
    if (far) {
      if (SEG) badsh(sh0); else atomicOr(&ds->fc.rare, 32u);
    } else if (pv < 0) {
      if (!SEG) ds->pos0 = T.p0;   // the stream's first candidate: ReadAll's first frame must be it (at 0)
      else if (!sfirst0) badsh(sh0);
    } else {
      const bool near = pv == (int64_t)t - 1;
      const uint64_t ppz = near ? P_pz : a.trec[pv].pz, psz = near ? P_sz : a.trec[pv].sz;
      const uint32_t pcrc = near ? P_crcz : a.trec[pv].crcz;
      const uint32_t psh = SEG ? pos_shard_in(sg.soff, 0, sg.ns, ppz) : 0u;
      if (!SEG || psh == sh0) {
        if (psz != T.p0) {
          if (SEG) badsh(sh0); else atomicOr(&ds->irregular, 1u);
        }
        if (!sfirst0) {
          seed0 = pcrc;
          seeded0 = true;
        }
      } else if (!sfirst0) {
        badsh(sh0);
      }
    }
    // ---- the first frame's check, its successor in the tile ----
    if ((T.flags & FRT_T0) && (T.flags & FRT_PE0) && !(T.flags & FRT_TORN0) && seeded0) {
      const int st = fr_check(s_n, a.g_shift, T.type0, T.crc0, seed0, T.pfd0, T.pe0, T.dlen0, false);
      if (st) key_at(sh0, T.p0, st);
    }
    SEAM_T(2);
    // ---- the last frame ----
    const uint32_t shz = SEG ? pos_shard_in(sg.soff, 0, sg.ns, T.pz) : 0u;
    const uint64_t EZ = SEG ? sg.soff[shz + 1] : a.B;
    const bool tornz = (T.flags & FRT_TORNZ) != 0;
    bool seededz = false;
    uint32_t seedz = 0;
    if (T.flags & FRT_SEEDZ) {
      seededz = true;
      seedz = T.seedz;
    } else if (T.count == 1 && (T.flags & FRT_T0)) {
      seededz = seeded0 && !far;
      seedz = seed0;
    }
    uint32_t nx = t + 1;
    sc = 0;
    bool farn = false;
    if (!(hn && cn)) {
      while (nx < a.ntiles && a.tcnt[nx] == 0) {
        if (++sc > FR_SCAN) { farn = true; break; }
        ++nx;
      }
    }
    const bool hasn = !farn && nx < a.ntiles;
    const uint64_t e = T.sz;   // canonical layout: the Data ends at the frame end
    uint32_t Pe = 0;
    bool pe_ok = false;
    if (farn) {
      if (SEG) badsh(shz); else atomicOr(&ds->fc.rare, 32u);
    } else if (hasn) {
      const bool nnear = nx == t + 1;
      const uint64_t np = nnear ? N_p0 : a.trec[nx].p0;
      const uint32_t nsh = SEG ? pos_shard_in(sg.soff, 0, sg.ns, np) : 0u;
      if (!SEG || nsh == shz) {
        if (np != T.sz) {
          if (SEG) badsh(shz); else atomicOr(&ds->irregular, 1u);
        }
      } else if (!tornz && T.sz != EZ) {   // the shard's last frame ends before the shard: the terminal
        const int tst = fr_terminal(a.buf, a.B, T.sz, EZ);
        if (tst < 0) badsh(shz);
        else atomicMin(&sg.sp[shz].term, (T.sz << 8) | (uint32_t)tst);
      }
      if (np == e) {
        const uint64_t tsn = (uint64_t)nx * TB;
        const uint32_t span = nnear ? T_agg : fr_span_lin(a.trec, t, nx, s_n, TLOG);
        Pe = seam_shift(s_n, a.g_shift, e - tsn, span) ^ (nnear ? N_pfo0 : a.trec[nx].pfo0);
        pe_ok = true;
      }
    } else {   // the stream's last frame
      if (!SEG) {
        ds->q = T.sz;
        ds->qlen = (T.sz <= a.B && a.B - T.sz >= 8) ? (int64_t)ld_le64_b(a.buf, a.B, T.sz) : 0;
        ds->fc.last_chained = T.crcz;
        // a whole frame at q the piece filter did not admit: the general path walks it (k_walk)
        if (!tornz && fr_terminal(a.buf, a.B, T.sz, a.B) < 0) atomicOr(&ds->fc.rare, 128u);
      } else if (!tornz && T.sz != EZ) {
        const int tst = fr_terminal(a.buf, a.B, T.sz, EZ);
        if (tst < 0) badsh(shz);
        else atomicMin(&sg.sp[shz].term, (T.sz << 8) | (uint32_t)tst);
      }
    }
    if (!pe_ok && !farn && T.dlenz && e <= a.B)   // (the stream's end: from the frame pass when it kept it)
      Pe = (e == a.B && (T.flags & FRT_PEB)) ? T.peB : fr_pe_far(a, s_n, t, e, TU, TLOG);
    if (!tornz && !farn && seededz && (T.flags & FRT_OKZ)) {
      const bool defer = !SEG && T.pz == 0 && ds->defer_first;
      const int st = fr_check(s_n, a.g_shift, T.typez, T.crcz, seedz, T.pfdz, Pe, T.dlenz, defer);
      if (st) key_at(shz, T.pz, st);
    }
    SEAM_T(3);
    // ---- the gap rule for the tile's first entry op (wal/wal.go:173) ----
    if (T.seam && T.nops) {
      const uint32_t shf = SEG ? pos_shard_in(sg.soff, 0, sg.ns, T.firstop_p) : 0u;
      const uint64_t ri = SEG ? sg.ri[shf] : a.ri;
      const uint64_t lo_p = SEG ? sg.soff[shf] : 0ull;
      bool has = false, farop = false;
      uint64_t pidx = 0;
      uint32_t scanned = 0;
      int64_t u0 = (int64_t)t - 1;
      if (hp && cp && P_nops && (uint64_t)t * TB > lo_p) {   // the previous tile holds the predecessor op
        has = !SEG || P_lastop >= lo_p;
        pidx = P_lastidx;
        u0 = -1;
      }
      for (int64_t u = u0; u >= 0 && (uint64_t)(u + 1) * TB > lo_p; --u) {
        if (++scanned > FR_SCAN) { farop = true; break; }
        if (!a.tcnt[u] || !a.trec[u].nops) continue;   // (a tile without frames has no op fields written)
        has = !SEG || a.trec[u].lastop_p >= lo_p;
        pidx = a.trec[u].last_index;
        break;
      }
      if (farop) {
        if (SEG) badsh(shf); else atomicOr(&ds->fc.rare, 32u);
      } else {
        const uint64_t k = T.first_index - ri;
        bool gap;
        if (has) {
          const uint64_t kq = pidx - ri;
          if (k <= kq) {
            if (SEG) sg.sp[shf].rew = (a.rew && sg.sp[shf].rmode) ? 2u : 1u;   // 2: its claims are in the pass
            else if (!a.rew) atomicOr(&ds->fc.rare, 2u);
            else atomicOr(&ds->fr_rews, 1u);
          }
          gap = k > kq && k - kq > 1;
        } else {
          gap = k > 0;
        }
        if (gap) key_at(shf, T.firstop_p, EWAL_PANIC_INDEX_GAP);
      }
    }
    if (!SEG) {
      fail = min(fail, T.fail);
      meta = min(meta, (unsigned long long)T.meta0);
      le = max(le, (unsigned long long)T.last_entry1);
      ls = max(ls, (unsigned long long)T.last_state1);
      if (T.nops) lo = max(lo, (unsigned long long)T.lastop_p + 1);
      nops += T.nops;
    }
  }
  SEAM_T(4);
#ifdef FR_TIMING
  if (threadIdx.x == 0 && blockIdx.x < 1024)
    for (int i = 0; i < 8; ++i) fr_sdbg2[blockIdx.x * 8 + i] = tq[i] ? tq[i] - tq[0] : 0ull;
  if (blockIdx.x < 1024)
    for (int i = 1; i < 5; ++i)
      if (tq[i]) atomicMax(&fr_sdbg3[blockIdx.x * 8 + i], tq[i] - tq[0]);   // cycles from the loop start
#endif
  if (SEG) return;
  // the block's fold: a wave reduction first, then one LDS atomic per wave
  for (int o = 32; o; o >>= 1) {
    fail = min(fail, (unsigned long long)__shfl_xor((long long)fail, o));
    meta = min(meta, (unsigned long long)__shfl_xor((long long)meta, o));
    le = max(le, (unsigned long long)__shfl_xor((long long)le, o));
    ls = max(ls, (unsigned long long)__shfl_xor((long long)ls, o));
    lo = max(lo, (unsigned long long)__shfl_xor((long long)lo, o));
    nops += (unsigned long long)__shfl_xor((long long)nops, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (fail != ~0ull) atomicMin(&s_red[0], fail);
    if (meta != ~0ull) atomicMin(&s_red[1], meta);
    if (le) atomicMax(&s_red[2], le);
    if (ls) atomicMax(&s_red[3], ls);
    if (lo) atomicMax(&s_red[4], lo);
    if (nops) atomicAdd(&s_red[5], nops);
  }
  __syncthreads();
#ifdef FR_TIMING
  const unsigned long long t_fold = clock64();
#endif
  if (threadIdx.x == 0) {
    if (s_red[0] != ~0ull) atomicMax(&ds->fc.fail_inv, ~s_red[0]);
    if (s_red[1] != ~0ull) atomicMax(&ds->fc.meta_inv, ~s_red[1]);
    if (s_red[2]) atomicMax(&ds->fr.le, s_red[2]);
    if (s_red[3]) atomicMax(&ds->fr.ls, s_red[3]);
    if (s_red[4]) atomicMax(&ds->fr.lo, s_red[4]);
    if (s_red[5]) atomicAdd(&ds->fr.nops, s_red[5]);
#ifndef FR_SEAM_NOFENCE   // (timing only: the fence's price; results may be stale without it)
    __threadfence();
#endif
    s_last = atomicAdd(&ds->fc_done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
#ifdef FR_TIMING
  const unsigned long long t_loop = clock64();
#endif
  if (s_last) {   // the last workgroup: every tile is in
    __threadfence();
    fr_result<TSH>(a, o, h, s_w, s_d, &s_ord, s_res);
  }
#ifdef FR_TIMING
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    fr_sdbg[blockIdx.x * 4 + 0] = t_loop - t_seam0;
    fr_sdbg[blockIdx.x * 4 + 1] = s_last ? clock64() - t_loop : 0ull;
    fr_sdbg[blockIdx.x * 4 + 2] = t_seam0;
    fr_sdbg[blockIdx.x * 4 + 3] = t_loop;
    fr_sdbg2[blockIdx.x * 8 + 5] = tq[0] - t_seam0;            // staging + the first barrier
    fr_sdbg2[blockIdx.x * 8 + 6] = tq[4] ? t_loop - tq[4] : 0ull;   // after thread 0's last tile: the block's wait + fold
    fr_sdbg2[blockIdx.x * 8 + 7] = t_loop - t_fold;                 // the block's device atomics, fence, done count
  }
#endif
}

// ewal_copy_range_info after a ReadAll the frame pass decided (no per-frame
// descriptors to run k_range_info over): the frames k_range_info names, from
// the pass's reductions -- the first metadata frame (the metadata list), the
// first non-empty one, the first entry op (the first tile with ops; no entry
// below ri met, so it is the first entry frame), the last entry / op / state
// frame -- and frame 0, each re-read (fc_frame_fields) with its ordinal
// (fr_ordinal).  One workgroup of 8 waves; hs = the pass's Small.
#define RFR_N 7   // md_first, md_value, ent_first, ent_last, op_last, st_last, frame 0
struct RangeFr {
  unsigned long long pos[RFR_N];   // stream position (~0: none)
  unsigned long long ord[RFR_N];
  RecDesc d[RFR_N];
  uint32_t u0, pad;                // frame 0: crc32.Update(0, Data) (the caller's check of a deferred frame 0)
};
template <int TSH>
__global__ __launch_bounds__(512) void k_range_info_fr(FrArgs a, uint32_t nmeta, unsigned long long meta_inv,
                                                       unsigned long long le, unsigned long long lo,
                                                       unsigned long long ls, unsigned long long K, RangeFr *o) {
  constexpr uint32_t TU = 1u << TSH;
  __shared__ unsigned long long s_pos[RFR_N];
  __shared__ uint4 s_w[RFR_N][6];
  __shared__ uint32_t s_n[SEAM_LDS];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  stage_lds<512>(s_n, SEAM_NIB * 128, [&](int i) { return nib_src(a.g_shift, i); });
  if (SEAM_DIG) stage_lds<512>(s_n + SEAM_NIB * 128, EW_DIG_TABS * 128, [&](int i) { return a.g_shift[EW_DIG_OFF + i]; });
  if (tid == 0) {
    s_pos[0] = ~0ull;
    s_pos[1] = meta_inv ? ~meta_inv : ~0ull;
    s_pos[3] = le ? le - 1 : ~0ull;
    s_pos[4] = lo ? lo - 1 : ~0ull;
    s_pos[5] = ls ? ls - 1 : ~0ull;
    s_pos[6] = K ? 0ull : ~0ull;
  }
  __syncthreads();
  unsigned long long mf = ~0ull;
  for (uint32_t i = tid; i < min(nmeta, a.mcap); i += blockDim.x) mf = min(mf, (unsigned long long)a.mlist[i]);
  for (int s = 32; s; s >>= 1) mf = min(mf, (unsigned long long)__shfl_xor((long long)mf, s));
  if (lane == 0 && mf != ~0ull) atomicMin(&s_pos[0], mf);
  if (wid == 7) {   // the first tile holding ops (count written for every tile, nops for tiles with frames)
    unsigned long long fp = ~0ull;
    for (uint32_t t0 = 0; t0 < a.ntiles; t0 += 64) {
      const uint32_t t = t0 + lane;
      const bool has = t < a.ntiles && a.tcnt[t] && a.trec[t].nops;
      const unsigned long long m = __ballot(has);
      if (m) {
        fp = a.trec[t0 + __ffsll((long long)m) - 1].firstop_p;
        break;
      }
    }
    if (lane == 0) s_pos[2] = fp;
  }
  __syncthreads();
  if (wid < RFR_N) {
    const unsigned long long x = s_pos[wid];
    unsigned long long ord = 0;
    if (x != ~0ull && wid != 6) ord = fr_ordinal(a, TU, x, nullptr);
    if (lane == 0) {
      o->pos[wid] = x;
      o->ord[wid] = ord;
      if (x != ~0ull) {
        const RecDesc f = fc_frame_fields(a.buf, a.B, x, s_w[wid]);
        o->d[wid] = f;
        if (wid == 6) {   // S_n(~0 ^ P(data start)) ^ P(data end) ^ ~0 (tile 0's prefixes are global)
          uint32_t u = 0;
          if (f.dlen)
            u = seam_shift(s_n, a.g_shift, f.dlen, 0xffffffffu ^ a.trec[0].pfd0) ^
                fr_pe_far(a, s_n, 0, f.doff + f.dlen, TU, 12 + TSH) ^ 0xffffffffu;
          o->u0 = u;
        }
      }
    }
  }
}

// Rewind mode: every listed slot (claimed by more than one entry op) gets
// the entry of its last op -- the one ReadAll's append leaves there (any op
// after it with a smaller index truncated below the slot and the ops after
// that climbed back through it, one index at a time).
__global__ __launch_bounds__(256) void k_ents_fix(const uint8_t *__restrict__ buf, uint64_t B,
                                                  const unsigned long long *__restrict__ own,
                                                  const uint32_t *__restrict__ clist, uint32_t ccap, const Small *ds,
                                                  ewal_entry *__restrict__ ents, const uint64_t *__restrict__ soff,
                                                  uint32_t ns) {
  __shared__ uint4 s_w[256][6];
  const uint32_t n = min(ds->fr_ncl, ccap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = clist[i];
    const uint64_t p = own[k] - 1;
    const RecDesc d = fc_frame_fields(buf, B, p, s_w[threadIdx.x]);
    const uint64_t base = soff ? soff[pos_shard_in(soff, 0, ns, p)] : 0ull;   // batch: Data relative to the shard
    ents[k] = ewal_entry{d.f0, d.f1, d.edoff - base, d.edlen, d.etype, (int32_t)d.enil};
  }
}

// ---- batch rewinds -------------------------------------------------------------
// A batched shard whose entry indexes go back (a leader change:
// ents = append(ents[:Index-ri], e), wal/wal.go:170-173) comes out of the
// batch's frame pass with every verdict field right -- the reductions are by
// stream position and a rewind is no gap -- except the ents slots written by
// more than one op: the waves store in no fixed order, and the slot must hold
// the LAST op's entry.  k_rew_claim walks the rewinding shards again at
// 64 KiB tiles (one wave per tile, many tiles per shard): the flagged pieces,
// the exact candidate tests, each candidate's canonical fields (no CRC, no
// prefixes -- the first pass checked them) and, per entry op, a claim of its
// slot with atomicMax(own, position + 1); the slots claimed twice are listed
// for k_ents_fix.  smask: the shards to claim for (1 byte each).
#define REW_TU 16   // units per claim tile (64 KiB)
__global__ __launch_bounds__(256) void k_rew_claim(const uint8_t *__restrict__ buf, uint64_t B, uint32_t nunits,
                                                   const ulonglong2 *__restrict__ hmask,
                                                   const uint32_t *__restrict__ tlist, uint32_t ntl,
                                                   const uint64_t *__restrict__ soff, uint32_t ns,
                                                   const uint64_t *__restrict__ ri, const uint64_t *__restrict__ rbase,
                                                   const uint8_t *__restrict__ smask,
                                                   unsigned long long *__restrict__ own, uint32_t *__restrict__ clist,
                                                   uint32_t ccap, Small *ds) {
  __shared__ uint4 s_w[256][6];
  const int lane = threadIdx.x & 63;
  const uint32_t wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  uint32_t over = 0;
  for (uint32_t ti = wid; ti < ntl; ti += nw) {   // (wave-uniform)
    const uint32_t u0 = tlist[ti] * REW_TU;
    const uint32_t u = u0 + (uint32_t)lane;
    const bool in = lane < REW_TU && u < nunits;
    const ulonglong2 h = in ? hmask[u] : make_ulonglong2(0ull, 0ull);
    const uint32_t c = (uint32_t)__popcll(h.x);
    const uint32_t incl = wave_incl_sum(c);
    const uint32_t Tf = rl32(incl, 63);
    for (uint32_t g0 = 0; g0 < Tf; g0 += 64) {
      const uint32_t g = g0 + (uint32_t)lane;
      const uint32_t gg = g < Tf ? g : Tf - 1;
      const int ol = owner_lane(incl, gg);
      const uint32_t r = gg - ((uint32_t)__shfl((int)incl, ol) - (uint32_t)__shfl((int)c, ol));
      const unsigned long long mx = shfl64(h.x, ol), m3 = shfl64(h.y, ol);
      if (g >= Tf) continue;
      const uint32_t pc = nth_bit(mx, r);
      const uint64_t poff = (uint64_t)(u0 + (uint32_t)ol) * EW_WAVE_BYTES + (uint64_t)pc * EW_PIECE;
      uint32_t D[19];
      if ((m3 >> pc) & 1ull) load_piece80(buf, B, poff, D);
      else load_piece64(buf, B, poff, D);
      const uint32_t fm = cand_filter(D);
      unsigned long long cm = fm ? cand_bits(D, fm, poff, B) : 0ull;
      while (cm) {
        const uint64_t p = poff + (uint64_t)__builtin_ctzll(cm);
        cm &= cm - 1;
        const uint32_t sh = pos_shard_in(soff, 0, ns, p);
        if (!smask[sh]) continue;
        const int64_t L = (int64_t)ld_le64_b(buf, B, p);
        if (L < 0 || p + 8 + (uint64_t)L > soff[sh + 1]) continue;   // torn: decoder.decode's terminal, no op
        const RecDesc d = fc_frame_fields(buf, B, p, s_w[threadIdx.x]);
        if (d.st || d.sub_st || d.type != 2 || d.f1 < ri[sh]) continue;
        const uint64_t k = d.f1 - ri[sh], rb = rbase[sh];
        if (k >= rbase[sh + 1] - rb) continue;
        if (atomicMax(&own[rb + k], (unsigned long long)(p + 1))) {   // a slot claimed twice
          const uint32_t ci = atomicAdd(&ds->fr_ncl, 1u);
          if (ci < ccap) clist[ci] = (uint32_t)(rb + k); else over = 1u;
        }
      }
    }
  }
  if (over) atomicOr(&ds->fc.rare, 64u);
}

// ---- batch (ewal_readall_batch_device) ----------------------------------------
// Per shard: the flagged pieces of the units overlapping it (an upper bound
// of its entry ops / 4: an entry frame is >= 20 bytes, so at most 4 of them
// start in one 64-B piece, and every frame start is a flagged piece).
__global__ __launch_bounds__(256) void k_shard_nfp(const ulonglong2 *__restrict__ hmask, uint32_t nunits,
                                                   const uint64_t *__restrict__ soff, uint32_t ns,
                                                   unsigned long long *__restrict__ nfp) {
  // one workgroup per shard (grid-strided): its units' flagged pieces summed, no atomics
  __shared__ unsigned long long s_sum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (uint32_t s = blockIdx.x; s < ns; s += gridDim.x) {
    const uint64_t b0 = soff[s], b1 = soff[s + 1];
    unsigned long long c = 0;
    if (b1 > b0) {
      const uint32_t ua = (uint32_t)(b0 >> 12), ub = (uint32_t)min<uint64_t>((b1 - 1) >> 12, (uint64_t)nunits - 1);
#pragma unroll 4
      for (uint32_t u = ua + (uint32_t)tid; u <= ub; u += blockDim.x) c += (unsigned long long)__popcll(hmask[u].x);
    }
    for (int o = 32; o; o >>= 1) c += (unsigned long long)__shfl_xor((long long)c, o);
    if (lane == 0) s_sum[wv] = c;
    __syncthreads();
    if (tid == 0) nfp[s] = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
    __syncthreads();
  }
}
// One workgroup: rbase[s] = 4 * (flagged pieces of the shards before s) --
// the ents region of shard s -- and the per-shard reductions initialised; a
// total past the capacity stops the frame pass (the host grows ents, reruns).
__global__ __launch_bounds__(1024) void k_shard_rbase(const unsigned long long *__restrict__ nfp, uint32_t ns,
                                                      uint64_t ecap, uint64_t *__restrict__ rbase,
                                                      ShardPos *__restrict__ sp, Small *ds) {
  __shared__ unsigned long long s_w[16];
  __shared__ unsigned long long s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < ns; c0 += 1024) {
    const uint32_t s = c0 + (uint32_t)tid;
    const unsigned long long x = s < ns ? 4ull * nfp[s] : 0ull;
    unsigned long long inc = x;
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = (unsigned long long)__shfl_up((long long)inc, d);
      if (lane >= d) inc += y;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    unsigned long long before = s_carry;
    for (int i = 0; i < wv; ++i) before += s_w[i];
    if (s < ns) {
      rbase[s] = before + inc - x;
      ShardPos p;
      p.first_fail = ~0ull;
      p.first_meta = ~0ull;
      p.term = ~0ull;
      p.last_entry = p.last_state = p.lastop = p.lastp = -1;
      p.bad = 0;
      p.open = 0;
      p.rew = 0;
      p.rmode = 0;
      sp[s] = p;
    }
    __syncthreads();
    if (tid == 1023) s_carry = before + inc;
    __syncthreads();
  }
  if (tid == 0) {
    rbase[ns] = s_carry;
    ds->fr_need = s_carry;
    if (s_carry > ecap) ds->fr_capfail = 1;
  }
}

// The listed shards' reductions initialised again (the rewind-mode pass
// over their tiles), and the pass's scratch counters.
__global__ void k_shard_reset(ShardPos *__restrict__ sp, const uint32_t *__restrict__ list, uint32_t n, Small *ds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    ds->fr_ncl = 0;
    ds->fr_tick = 0;
    ds->fc.rare = 0;
  }
  if (i >= n) return;
  ShardPos p;
  p.first_fail = ~0ull;
  p.first_meta = ~0ull;
  p.term = ~0ull;
  p.last_entry = p.last_state = p.lastop = p.lastp = -1;
  p.bad = 0;
  p.open = 0;
  p.rew = 0;
  p.rmode = 1;
  sp[list[i]] = p;
}

// The shards a ctx's previous batch saw rewind (list[0..n)) run this batch's
// frame pass in rewind mode: their ops claim their slots (FrArgs.own) and
// k_ents_fix rewrites the slots claimed twice right after the pass -- no
// second pass over their tiles.  After k_shard_rbase: rmode set, the shards'
// own[] regions unclaimed (one workgroup per listed shard, grid-strided).
__global__ __launch_bounds__(256) void k_shard_hint(ShardPos *__restrict__ sp, const uint32_t *__restrict__ list,
                                                    uint32_t n, const uint64_t *__restrict__ rbase,
                                                    unsigned long long *__restrict__ own, const Small *ds) {
  if (ds->fr_capfail) return;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t s = list[i];
    if (threadIdx.x == 0) sp[s].rmode = 1u;
    for (uint64_t k = rbase[s] + threadIdx.x; k < rbase[s + 1]; k += blockDim.x) own[k] = 0ull;
  }
}

// One workgroup: tcb[t] = candidates of the tiles before t.
__global__ __launch_bounds__(1024) void k_tile_scan(const uint32_t *__restrict__ tcnt, uint32_t nt, uint32_t *__restrict__ tcb,
                                                    const Small *ds) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_carry;
  if (ds->fr_capfail) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nt; c0 += 1024) {
    const uint32_t t = c0 + (uint32_t)tid;
    const uint32_t x = t < nt ? tcnt[t] : 0u;
    const uint32_t inc = wave_incl_sum(x);
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t before = s_carry;
    for (int i = 0; i < wv; ++i) before += s_w[i];
    if (t < nt) tcb[t] = before + inc - x;
    __syncthreads();
    if (tid == 1023) s_carry = before + inc;
    __syncthreads();
  }
}

// Per shard: ReadAll's metadata rule over the listed metadata frames.
__global__ void k_meta_batch_fr(FrArgs a, FrSeg sg) {
  __shared__ uint4 s_w[256][6];
  const Small *ds = a.ds;
  if (ds->fr_capfail || ds->fc.rare) return;
  const uint32_t nm = ds->nmeta;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nm; i += gridDim.x * blockDim.x) {
    const uint64_t p = a.mlist[i];
    const uint32_t s = pos_shard_in(sg.soff, 0, sg.ns, p);
    const unsigned long long fm = sg.sp[s].first_meta;
    if (fm == ~0ull || p <= fm) continue;
    const RecDesc d = fc_frame_fields(a.buf, a.B, p, s_w[threadIdx.x]);
    const RecDesc m = fc_frame_fields(a.buf, a.B, fm, s_w[threadIdx.x]);
    bool eq = d.dlen == m.dlen;
    for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = a.buf[d.doff + k] == a.buf[m.doff + k];
    if (!eq) atomicMin(&sg.sp[s].first_fail, (p << 8) | EWAL_ERR_METADATA_CONFLICT);
  }
}

// Per shard (one wave): its ReadAll result.  Ordinals from positions
// (fr_ordinal with the tile prefix); the frames the result names re-read by
// lanes 0..5.
template <int TSH>
__global__ __launch_bounds__(256) void k_result_batch_fr(FrArgs a, FrSeg sg, ewal_result *__restrict__ out,
                                                         unsigned long long *__restrict__ ent_first) {
  __shared__ uint4 s_w[256][6];
  __shared__ RecDesc s_d[256];
  const Small *ds = a.ds;
  if (ds->fr_capfail || ds->fc.rare) return;   // (a void pass: the host discards out[])
  const int lane = threadIdx.x & 63;
  const uint32_t s = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (s >= sg.ns) return;   // (wave-uniform)
  const ShardPos A = sg.sp[s];
  const uint64_t so = sg.soff[s], se = sg.soff[s + 1], ri = sg.ri[s];
  const uint32_t tu = 1u << TSH;
  const uint64_t f0 = fr_ordinal(a, tu, so, sg.tcb);
  const uint64_t fE = fr_ordinal(a, tu, se, sg.tcb);
  const uint64_t q = A.term != ~0ull ? (A.term >> 8) : se;
  const uint64_t f1 = A.term != ~0ull ? fr_ordinal(a, tu, q, sg.tcb) : fE;
  const uint64_t pf = A.first_fail != ~0ull ? (A.first_fail >> 8) : se;
  const uint64_t ff = A.first_fail != ~0ull ? fr_ordinal(a, tu, pf, sg.tcb) : 0;
  long long fr = -1;
  switch (lane) {
  case 0: fr = A.first_fail != ~0ull ? (long long)pf : -1; break;
  case 1: fr = A.last_entry; break;
  case 2: fr = A.lastp; break;
  case 3: fr = A.first_meta != ~0ull ? (long long)A.first_meta : -1; break;
  case 4: fr = A.last_state; break;
  case 5: fr = A.lastop; break;
  default: break;
  }
  if (fr >= 0) s_d[threadIdx.x] = fc_frame_fields(a.buf, a.B, (uint64_t)fr, s_w[threadIdx.x]);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane != 0) return;
  const RecDesc *D = s_d + threadIdx.x;
  ewal_result o;
  memset(&o, 0, sizeof(o));
  o.fail_record = -1;
  o.fail_offset = -1;
  o.metadata_off = -1;
  o.n_records = (int64_t)(f1 - f0);
  o.n_candidates = (int64_t)(fE - f0);
  o.n_runs = 1;
  unsigned long long ef = 0;
  const int tst = A.term != ~0ull ? (int)(A.term & 0xff) : EWAL_OK;
  if (A.first_fail != ~0ull) {
    o.status = (int32_t)(A.first_fail & 0xff);
    o.fail_record = (int64_t)(ff - f0);
    o.fail_offset = (int64_t)(pf - so);
    o.n_records = o.fail_record;
    if (o.status == EWAL_ERR_UNEXPECTED_TYPE) o.detail = D[0].type;
    if (o.status == EWAL_PANIC_INDEX_GAP) o.detail = (int64_t)D[0].f1;
  } else if (tst != EWAL_OK) {   // ReadAll returns decoder.decode's error (wal/wal.go:197-201)
    o.status = tst;
    o.fail_record = (int64_t)(f1 - f0);
    o.fail_offset = (int64_t)(q - so);
  } else {
    const uint64_t enti = A.last_entry >= 0 ? D[1].f1 : 0;
    o.enti = enti;
    if (enti < ri) {
      o.status = EWAL_ERR_INDEX_NOT_FOUND;
    } else if (f1 > f0) {
      // the running CRC after the shard's last frame: its stored CRC (a
      // verified frame's computed CRC equals it; crcType re-seeds to it)
      o.last_crc = D[2].crc;
      if (A.first_meta != ~0ull) {
        o.metadata_off = (int64_t)(D[3].doff - so);
        o.metadata_len = (int64_t)D[3].dlen;
      }
      if (A.last_state >= 0) {
        o.has_state = 1;
        o.state_term = D[4].f0;
        o.state_vote = D[4].f1;
        o.state_commit = D[4].f2;
      }
      o.n_ents = A.lastop >= 0 ? (int64_t)(D[5].f1 - ri + 1) : 0;
      ef = o.n_ents ? sg.rbase[s] : 0;   // op k of the shard is ents[rbase[s] + k]
    }
  }
  o.flags = EWAL_FLAG_FAST_PATH;
  if (A.rew == 1) o.flags |= EW_SHARD_REW;                      // the rewind-mode pass over its tiles
  if (A.rew == 2) o.flags |= EW_SHARD_REWIN;                    // resolved in this pass (rmode: claims + k_ents_fix)
  if (A.bad || (se > so && !A.open)) o.flags = EW_SHARD_BAD;   // replayed alone by the host
  out[s] = o;
  ent_first[s] = ef;
}

// The batch's verdict (one thread): spec_n = frames when the pass decided
// (shards it could not decide carry EW_SHARD_BAD), else 0; Small -> host.
__global__ void k_batch_gate_fr(Small *ds, Small *h) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t K = ds->total;
  const bool ok = !ds->fr_capfail && !ds->fc.rare && !ds->errflag && K < 0xffffff00ull;
  ds->spec_n = ok ? (uint32_t)(K ? K : 1) : 0u;
  *h = *ds;
}
