// fused_kernels.hip -- the regular-path frame pass fused with the chained CRC
// check.  ONE kernel (k_fc) decodes every frame, checks its CRC against its
// predecessor's stored CRC, applies ReadAll's per-frame rules and places the
// entry ops in ents, so the per-frame descriptors (RecDesc: 96 B written by
// k_frame and read back by k_check, plus the 8 B of prefixes) never touch
// HBM, and two launches (k_spec_gate, k_decode_slow) disappear.
//
// Reference: (*WAL).ReadAll wal/wal.go:164-216, decoder.decode
// wal/decoder.go:28-47, walpb.Record.Unmarshal wal/walpb/record.pb.go:43-136,
// raftpb.Entry / HardState.Unmarshal raft/raftpb/raft.pb.go:170-277, 618-704.
//
// k_fc decides the regular case: the candidates form one chain from byte 0,
// every frame is in the canonical encoding etcd's encoder writes, and entry
// indexes never rewind.  Anything else sets Small.irregular / Small.fc.rare
// and the host runs the general path (k_frame, k_decode_slow, k_check, the
// op-list passes) over the same stream pass -- nothing is guessed.
//
// Frames are processed in tiles of FC_TILE = 64 consecutive frames, one
// frame per lane, each tile by ONE wave: a persistent grid of FC_WGS
// workgroups per CU shares the LDS tables, and every wave then runs its own
// tiles (wave w: tiles w, w + all waves, ...) with no workgroup barrier, so
// the waves hide each other's memory latency.  Within a tile the
// predecessor's stored CRC and the successor's prefix come from the
// neighbouring lane (wave shuffles); the tile's edge frames are checked by
// k_fc_seam from the neighbouring tiles' records, which also folds the
// tiles' reductions.  Entry ops need no global
// numbering: in the regular case (no index gap -- a panic -- and no rewind --
// the general path) op k of a WAL has Index - ri == k, so each op goes
// straight to ents[Index - ri] (batched: the shard's region starts at its
// first frame, fs[s], and never holds more ops than the shard has frames).
// The index-gap rule for a tile's FIRST op, whose predecessor op lives in an
// earlier tile, is applied by k_fc_seam from the tiles' records (the nearest
// earlier tile with ops holds the predecessor's Index).
#include "ewal_device.h"
#include "ewal_internal.h"

// The single WAL's ents are written with nontemporal stores (40 B per op,
// read back only by the host's copy or the next call): configs[1]
// post-stream -8 us; the batched path keeps plain stores (+1-2 % with
// nontemporal ones, profiles/r02/ab_nt_ents.txt).
__device__ __forceinline__ void store_entry_nt(ewal_entry *dst, const ewal_entry &e) {
  uint64_t *q = (uint64_t *)dst;
  __builtin_nontemporal_store(e.term, q);
  __builtin_nontemporal_store(e.index, q + 1);
  __builtin_nontemporal_store(e.data_off, q + 2);
  __builtin_nontemporal_store(e.data_len, q + 3);
  __builtin_nontemporal_store(((uint64_t)(uint32_t)e.data_nil << 32) | (uint32_t)e.type, q + 4);
}

#ifndef FC_THREADS
#define FC_THREADS 256
#endif
#define FC_WAVES (FC_THREADS / 64)
#ifndef FC_WGS
#define FC_WGS 3          // resident workgroups per CU (LDS ~49 KiB each)
#endif
#define FC_OCC (FC_WGS * FC_WAVES / 4)   // waves per SIMD (the VGPR budget: 512 / FC_OCC)
#define FC_TILE 64        // frames per tile: one wave's, no workgroup barrier in the frame loop

// Per tile, for k_fc_seam: its entry ops (count, frames and Index of the
// first / last), the edge frames' CRC operands.
struct TileRec {
  uint32_t count;
  uint32_t first_frame, last_frame;   // of its first / last op
  uint32_t seam;       // 1: k_fc_seam applies the gap rule to the tile's first op
  uint64_t first_index, last_index;   // Index of its first / last op
  uint32_t lastcrc;    // the stored CRC of the tile's last frame (the next tile's first seed)
  uint32_t pfo0;       // P at the tile's first frame start (the previous tile's last P(data end))
  // the CRC checks k_fc leaves to k_fc_seam: [0] the tile's first frame
  // (seed: the frame before the tile), [1] its last frame (P(data end): the
  // next tile's first frame start); same frame when the tile has one frame
  uint32_t dfirst, dlast;
  uint32_t crc[2], pfd[2], seed1, pe0;
  int32_t type[2];
  uint64_t dlen[2];
  // the tile's reductions (single WAL; k_fc_seam folds them)
  unsigned long long fail;        // min (frame << 8 | status), ~0: none
  uint32_t last_entry1, last_state1, meta1, lastop1;   // 1 + frame (0: none); meta1: the first metadata frame
};

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

// k_fc ran over every frame (its tile records, ents and mlist are filled):
// what the kernels after it need before they read them.
__device__ __forceinline__ bool fc_ran(const Small *ds, uint64_t ccap, uint64_t ecap) {
  const uint64_t K = ds->total;
  return K && K <= ccap && K <= ecap && K < 0xffffff00ull && !ds->novf && !ds->errflag;
}
// ... and decided the regular case (the results are the reference's).
__device__ __forceinline__ bool fc_valid(const Small *ds, uint64_t ccap, uint64_t ecap) {
  return fc_ran(ds, ccap, ecap) && ds->pos0 == 0 && !ds->irregular && !ds->fc.rare;
}
// Batched: the regular case is decided per shard (ShardAgg.bad: a shard whose
// frames are not its candidates, or that needs a rare path, is replayed alone
// by the host); what stays global is capacity.
__device__ __forceinline__ bool fc_valid_seg(const Small *ds, uint64_t ccap, uint64_t ecap) {
  return fc_ran(ds, ccap, ecap) && !ds->fc.rare;
}

// S_{2^m} as nibble tables: N[m][k][d] = S_{2^m}(d << 4k), 8 x 16 entries per
// operator (512 B; m = 0..16 in 8.5 KiB of LDS instead of 68 KiB of byte
// tables), 8 lookups per application.
#define FC_NIB_LEVELS 17
__device__ __forceinline__ uint32_t nib_src(const uint32_t *g_shift, int i) {
  const int m = i >> 7, k = (i >> 4) & 7, d = i & 15;
  return g_shift[m * 1024 + (k >> 1) * 256 + (d << (4 * (k & 1)))];
}


struct FcArgs {
  const uint8_t *buf;
  uint64_t B;
  const uint64_t *cpos;
  uint64_t ccap;        // capacity of the candidate list
  uint64_t ecap;        // capacity of ents / mlist
  const uint32_t *pwave, *v, *g_slice, *g_shift;
  uint64_t ri;          // w.ri (single WAL)
  TileRec *trec;
  ewal_entry *ents;
  uint32_t *mlist;
  Small *ds;
  uint32_t ablate;      // EWAL_FC_ABLATE timing experiments only (results are wrong): 1 shift, 2 prefixes,
                        // 4 look-back, 8 ents stores, 16 no failure reports
};

// walpb.Record's stored Crc from a canonical frame head at p (08 type 10
// crc): the tile's first frame takes its seed from it.  *ok clears when the
// head is not canonical (that frame's own tile reports it rare anyway).
__device__ __forceinline__ uint32_t fc_head_crc(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p, bool *ok) {
  uint8_t h[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) h[i] = (p + 8 + i < B) ? buf[p + 8 + i] : 0;
  int o = 0;
  bool good = h[o++] == 0x08;
  while (o < 12 && (h[o] & 0x80)) ++o;   // type varint
  ++o;
  good = good && o < 12 && h[o++] == 0x10;
  uint64_t c = 0;
  for (uint32_t sh = 0; o < 24; sh += 7) {
    const uint8_t b = h[o++];
    if (sh < 32) c |= (uint64_t)(b & 0x7f) << sh;
    if (b < 0x80) break;
  }
  *ok = good;
  return (uint32_t)c;
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
// memory (the passes after k_fc touch a handful of frames): Record type /
// crc / Data, Entry / HardState fields.  The first 96 bytes come in with six
// vector loads into this thread's LDS slot w (96 B), the walkers read the
// rest (if any) from global memory.
__device__ RecDesc fc_frame_fields(const uint8_t *__restrict__ buf, uint64_t B, uint64_t p, uint4 *w) {
  RecDesc d;
  d.off = p;
  d.type = 0; d.crc = 0; d.chained = 0; d.st = 0; d.sub_st = 0;
  d.doff = p + 8; d.dlen = 0; d.dnil = 1;
  d.f0 = d.f1 = d.f2 = 0; d.edoff = 0; d.edlen = 0; d.enil = 1; d.etype = 0; d.pad0 = 0; d.pad1 = 0;
  const int64_t L = (int64_t)ld_le64_b(buf, B, p);
  if (p + 8 > B || L < 0 || (uint64_t)L > B - p - 8) {   // not a frame (only a void pass asks)
    d.st = EWAL_ERR_UNEXPECTED_EOF;
    return d;
  }
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

template <bool SEG>
__global__ __launch_bounds__(FC_THREADS, FC_OCC) void k_fc(FcArgs a, SegArgs sg) {
  __shared__ uint32_t s_t4[16 * 256];          // slicing-by-16
  __shared__ uint32_t s_svp[1024];             // S_256 (prefix Horner step)
  __shared__ uint32_t s_nib[FC_NIB_LEVELS * 128];   // S_{2^0} .. S_{2^16}, nibble tables (the seed shift)
  __shared__ uint32_t s_inv[7 * 128];               // S_{2^0}^-1 .. S_{2^6}^-1 (prefixes from the next boundary)
  __shared__ uint32_t s_win[20 * FC_THREADS];  // frame heads, transposed (bank = thread & 31)
  Small *ds = a.ds;
  const uint64_t K = ds->total;
  if (K == 0 || K > a.ccap || ds->novf || K >= 0xffffff00ull) return;   // the host takes the general path
  if (K > a.ecap) {                           // no room for every op: the host grows ents, once
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&ds->fc.rare, 4u);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t K32 = (uint32_t)K;
  const uint32_t ntiles = (K32 + FC_TILE - 1) / FC_TILE;
  const uint32_t wid = blockIdx.x * FC_WAVES + (uint32_t)(tid >> 6), nwaves = gridDim.x * FC_WAVES;
  uint32_t rare = 0, irr = 0;
  // this lane's candidate offsets, one tile ahead
  auto cand = [&](uint32_t tt, uint64_t &pp, uint64_t &pq) {
    const uint32_t rr = min(tt * FC_TILE + (uint32_t)lane, K32 - 1);
    pp = a.cpos[rr];
    pq = rr + 1 < K32 ? a.cpos[rr + 1] : ~0ull;
  };
  uint64_t p_nx = 0, pn_nx = 0;
  // single WAL: tiles grid-strided over the waves; batched: each wave takes
  // a contiguous run of tiles, so consecutive tiles mostly share a shard and
  // its reductions are folded in registers (one set of atomics per run of
  // tiles in one shard instead of per tile: ~10 % of this pass at 128 shards)
  const uint32_t chunk = (ntiles + nwaves - 1) / nwaves;
  const uint32_t tbeg = SEG ? min(wid * chunk, ntiles) : wid;
  const uint32_t tend = SEG ? min(tbeg + chunk, ntiles) : ntiles;
  const uint32_t tstep = SEG ? 1u : nwaves;
  if (tbeg < tend) cand(tbeg, p_nx, pn_nx);   // in flight while the tables are staged
  stage_lds<FC_THREADS>(s_t4, 16 * 256, [&](int i) { return a.g_slice[i]; });
  stage_lds<FC_THREADS>(s_svp, 1024, [&](int i) { return a.g_shift[EW_VLOG * 1024 + i]; });
  stage_lds<FC_THREADS>(s_nib, FC_NIB_LEVELS * 128, [&](int i) { return nib_src(a.g_shift, i); });
  stage_lds<FC_THREADS>(s_inv, 7 * 128, [&](int i) { return nib_src(a.g_shift + EW_SHIFT_LEVELS * 1024, i); });
  __syncthreads();   // the only barrier: every wave runs its own tiles from here on
  // SEG: the shard of the run's first tile, one search per wave (binary
  // searches per tile were chains of dependent loads on every tile)
  uint32_t scur = (SEG && tbeg < tend) ? shard_of(sg.fs, sg.ns, tbeg * FC_TILE) : 0u;
  uint32_t ash = EW_NIL, alo = 0;                 // SEG: the shard folded so far and its reductions
  unsigned long long aff = ~0ull, afm = ~0ull;
  long long ale = -1, als = -1;
  auto aflush = [&]() {
    if (ash != EW_NIL && lane == 0) {
      ShardAgg *A = sg.sagg + ash;
      if (aff != ~0ull) atomicMin(&A->first_fail, aff);
      if (ale >= 0) atomicMax(&A->last_entry, ale);
      if (als >= 0) atomicMax(&A->last_state, als);
      if (afm != ~0ull) atomicMin(&A->first_meta, afm);
      if (alo) atomicMax(&A->lastop, alo);
    }
    aff = afm = ~0ull;
    ale = als = -1;
    alo = 0;
  };
  ewal_entry pe;      // the ents store held over to the next tile (below)
  uint64_t pidx = 0;
  bool pend = false;
  if (wid == 0 && lane == 0) ds->pos0 = a.cpos[0];
  for (uint32_t t = tbeg; t < tend; t += tstep) {
    const uint32_t r0 = t * FC_TILE;
    const uint32_t rt = r0 + (uint32_t)lane;
    const bool live = rt < K32;
    const uint32_t r = live ? rt : K32 - 1;    // writes masked for lanes past the end
    const uint32_t rl = min(r0 + FC_TILE, K32) - 1;   // the tile's last frame
    const uint64_t p = p_nx, pn = pn_nx;
    if (t + tstep < tend) cand(t + tstep, p_nx, pn_nx);
    RecDesc d;
    int64_t L = 0;
    uint32_t Pfo = 0, Pfd = 0;
    // the previous tile's ents store goes out behind this tile's loads (a
    // store issued before them would be waited for with them: vmcnt counts
    // loads and stores in order)
    auto flush = [&]() {
      if (pend) {
        if (SEG) a.ents[pidx] = pe;
        else store_entry_nt(a.ents + pidx, pe);
      }
      pend = false;
    };
    const bool ok = decode_canon<FC_THREADS, true>(a.buf, a.B, p, a.pwave, a.v, s_t4, s_svp, s_win + tid, d, L, Pfo,
                                                   Pfd, (a.ablate & 2) != 0, flush, s_inv);
    const uint64_t s = p + 8 + (uint64_t)L;
    uint32_t sh = 0, lo = 0;                   // SEG: the frame's shard and its first frame
    uint64_t ri = a.ri;
    uint32_t sh0 = 0, sh1 = 0;
    if (SEG) {   // the tile's shard range: the wave's run of tiles walks the shards forward
      while (scur + 1 < sg.ns && sg.fs[scur + 1] <= r0) ++scur;   // (uniform; usually no step)
      sh0 = scur;
      sh1 = sh0;
      while (sh1 + 1 < sg.ns && sg.fs[sh1 + 1] <= rl) ++sh1;
      sh = sh0 == sh1 ? sh0 : shard_in(sg.fs, sh0, sh1 + 1, r);
      lo = sg.fs[sh];
      ri = sg.ri[sh];
    }
    bool bad = false;   // SEG: this frame takes its shard off the regular path (the host replays it alone)
    // SEG: the shard's last candidate runs past the shard's end -- a torn
    // tail (a crash mid-write): decoder.decode stops at its length prefix
    // (io.ReadFull short, wal/decoder.go:30-36), so it is no frame of the
    // shard; the shard's verdict is its terminal's (classify below)
    const bool torn = SEG && live && r + 1 == sg.fs[sh + 1] && s > sg.soff[sh + 1];
    if (live && !ok && !torn) {
      if (SEG) bad = true;
      else rare |= 1u;
    }
    if (!ok) {   // not decoded (the pass is void): no field of it may address memory
      d.type = 0;
      d.dlen = 0;
      d.doff = p + 8;
    }
    if (SEG) {
      // a shard's frames are its candidates, the last one ending at the
      // shard's end -- or at decoder.decode's terminal inside it (a torn tail:
      // fewer than 8 bytes, or a length the bytes left cannot hold)
      if (live && r + 1 == sg.fs[sh + 1] && s != sg.soff[sh + 1]) {
        const uint64_t E = sg.soff[sh + 1];
        const uint64_t q = torn ? p : s;   // where the terminal sits
        int tst;
        if (E - q < 8) {
          tst = EWAL_ERR_UNEXPECTED_EOF;
        } else {
          const int64_t Lq = torn ? L : (int64_t)ld_le64_b(a.buf, a.B, q);
          const uint64_t rem = E - q - 8;
          if (Lq < 0) tst = EWAL_PANIC_NEG_LENGTH;
          else if ((uint64_t)Lq > rem) tst = rem == 0 ? EWAL_OK : EWAL_ERR_UNEXPECTED_EOF;
          else tst = -1;   // a frame that fits but is no candidate: the general walk
        }
        if (tst < 0) {
          bad = true;
        } else {
          ShardAgg *A = sg.sagg + sh;
          A->term1 = (torn ? r : r + 1) + 1u;
          A->term_st = tst;
          A->term_off = q;
        }
      } else if (live && r + 1 < sg.fs[sh + 1] && pn != s) {
        bad = true;
      }
    } else {
      if (live && r + 1 < K32 && pn != s) irr = 1;
      if (live && r + 1 == K32) {   // the chain's terminal
        ds->q = s;
        ds->qlen = (s <= a.B && a.B - s >= 8) ? (int64_t)ld_le64_b(a.buf, a.B, s) : 0;
      }
    }
    // neighbours in the wave: the predecessor's stored CRC, the successor's
    // P at its frame start; the tile's edge frames take theirs from the
    // neighbouring tiles' records in k_fc_seam
    const uint32_t cprev = (uint32_t)__shfl_up((int)d.crc, 1);
    const uint32_t pnext = (uint32_t)__shfl_down((int)Pfo, 1);
    // decoder.decode's check + ReadAll's crc-record rule (as k_check)
    const bool dfirst = lane == 0 && r > lo && !torn;
    const bool dlast = live && r == rl && r + 1 < K32 && !torn;
    const uint32_t seed = r > lo ? cprev : 0u;
    int st = 0;
    uint32_t chained = seed;
    uint32_t Pe = 0;
    if (d.type == 4) {
      if (seed != 0 && d.crc != seed) st = EWAL_ERR_WAL_CRC;
      chained = d.crc;
    } else {
      uint32_t computed = seed;
      if (d.dlen) {
        const uint64_t e = d.doff + d.dlen;
        // P(data end) = the successor's P at its frame start (canonical
        // layout), else computed here (the chain's last frame)
        Pe = pnext;
        if (!(e == pn && r + 1 < K32)) Pe = prefix_at(e, a.pwave, a.v, a.buf, s_t4, s_svp);
        if (dlast) Pe = 0;   // the next tile's (k_fc_seam)
        uint32_t x = seed ^ 0xffffffffu ^ Pfd;
        uint64_t m = d.dlen;
        if (!(a.ablate & 1))
          for (int lvl = 0; m; ++lvl, m >>= 1)
            if (m & 1) x = lvl < FC_NIB_LEVELS ? nib_apply(s_nib + lvl * 128, x) : gshift_pow2(a.g_shift, lvl, x);
        computed = x ^ Pe ^ 0xffffffffu;
      }
      chained = computed;
      // a range split inside a file (ewal_readall_range_device): frame 0's
      // Validate is the caller's -- the running CRC before it is not known here
      const bool defer0 = !SEG && r == 0 && ds->defer_first;
      if (computed != d.crc && !defer0) st = EWAL_ERR_RECORD_CRC;
      else if (d.type != 1 && d.type != 2 && d.type != 3) st = EWAL_ERR_UNEXPECTED_TYPE;
      if (defer0) chained = d.crc;   // the running CRC after it, once the caller's check holds
    }
    TileRec *tr = a.trec + t;
    if (live && (lane == 0 || r == rl)) {
      const int32_t ty = (int32_t)(d.type < 0 || d.type > 1000 ? 1000 : d.type);
      if (lane == 0) {
        tr->pfo0 = Pfo;
        tr->dfirst = dfirst;
        tr->crc[0] = d.crc;
        tr->pfd[0] = Pfd;
        tr->pe0 = Pe;
        tr->type[0] = ty;
        tr->dlen[0] = d.dlen;
      }
      if (r == rl) {   // the tile's last frame
        tr->lastcrc = d.crc;
        tr->dlast = dlast;
        tr->crc[1] = d.crc;
        tr->pfd[1] = Pfd;
        tr->seed1 = seed;
        tr->type[1] = ty;
        tr->dlen[1] = d.dlen;
      }
    }
    if (a.ablate & 16) st = 0;   // timing only: no failure reports (keeps the ablations' verdict path alike)
    if (torn) {   // no frame of its shard: no verdict, no type, no op
      st = 0;
      d.type = 0;
    }
    if (dfirst || dlast) st = 0;
    else if (live && r + 1 == K32) ds->fc.last_chained = chained;
    // entry ops (wal/wal.go:170-176): the op's predecessor in the tile; the
    // tile's first op is k_fc_seam's unless the tile opens its shard
    const bool op = live && d.type == 2 && d.f1 >= ri;
    const unsigned long long mo = __ballot(op);
    const unsigned long long below = mo & ((1ull << lane) - 1ull);
    unsigned long long bsh = below;
    if (SEG && lo > r0) bsh = (lo - r0 >= 64) ? 0ull : below & ~((1ull << (lo - r0)) - 1ull);
    const int pl = bsh ? 63 - __clzll((long long)bsh) : lane;
    const uint64_t kp = __shfl(d.f1, pl);
    const int wl = mo ? 63 - __clzll((long long)mo) : 0;
    const int wf = mo ? __ffsll((long long)mo) - 1 : 0;
    const uint64_t wli = __shfl(d.f1, wl), wfi = __shfl(d.f1, wf);
    const uint32_t ff = mo ? r0 + (uint32_t)wf : EW_NIL;
    bool tseam = mo != 0;
    if (SEG && mo) {   // the first op's shard began before the tile (one lane searches)
      int b = 0;
      if (lane == 0) b = sg.fs[shard_in(sg.fs, sh0, sh1 + 1, ff)] < r0;
      tseam = __shfl(b, 0) != 0;
    }
    // reductions: per tile into its record (k_fc_seam folds the tiles'),
    // batched: per shard (lane by lane where a shard starts inside the tile)
    const unsigned long long mf = __ballot(live && st != 0), me = __ballot(live && d.type == 2),
                             ms = __ballot(live && d.type == 3), mm = __ballot(live && d.type == 1 && d.dlen > 0);
    const int ffl = mf ? __ffsll((long long)mf) - 1 : 0;
    const uint32_t fst = (uint32_t)__shfl(st, ffl);
    if (live && d.type == 1 && st == 0) {     // ReadAll's metadata rule runs after the pass
      const uint32_t mi = atomicAdd(&ds->nmeta, 1u);
      if (mi < a.ecap) a.mlist[mi] = r; else rare |= 4u;
    }
    if (lane == 0) {
      tr->count = (uint32_t)__popcll(mo);
      tr->first_frame = ff;
      tr->last_frame = mo ? r0 + (uint32_t)wl : EW_NIL;
      tr->first_index = wfi;
      tr->last_index = wli;
      tr->seam = tseam;
      tr->fail = mf ? ((unsigned long long)(r0 + (uint32_t)ffl) << 8) | fst : ~0ull;
      tr->last_entry1 = me ? r0 + (uint32_t)(63 - __clzll((long long)me)) + 1u : 0u;
      tr->last_state1 = ms ? r0 + (uint32_t)(63 - __clzll((long long)ms)) + 1u : 0u;
      tr->meta1 = mm ? r0 + (uint32_t)(__ffsll((long long)mm) - 1) + 1u : 0u;
      tr->lastop1 = mo ? r0 + (uint32_t)wl + 1u : 0u;
    }
    if (SEG) {
      if (sh0 == sh1) {   // folded into the wave's run (wave-uniform values), flushed when the shard changes
        if (sh0 != ash) {
          aflush();
          ash = sh0;
        }
        if (mf) aff = min(aff, ((unsigned long long)(r0 + (uint32_t)ffl) << 8) | fst);
        if (me) ale = max(ale, (long long)(r0 + (uint32_t)(63 - __clzll((long long)me))));
        if (ms) als = max(als, (long long)(r0 + (uint32_t)(63 - __clzll((long long)ms))));
        if (mm) afm = min(afm, (unsigned long long)(r0 + (uint32_t)(__ffsll((long long)mm) - 1)));
        if (mo) alo = max(alo, r0 + (uint32_t)wl + 1u);
      } else if (live) {   // a shard boundary inside the tile (rare): lane by lane
        ShardAgg *A = sg.sagg + sh;
        if (st != 0) atomicMin(&A->first_fail, ((unsigned long long)r << 8) | (uint32_t)st);
        if (d.type == 2) atomicMax(&A->last_entry, (long long)r);
        if (d.type == 3) atomicMax(&A->last_state, (long long)r);
        if (d.type == 1 && d.dlen > 0) atomicMin(&A->first_meta, (unsigned long long)r);
        if (op) atomicMax(&A->lastop, r + 1u);
      }
    }
    if (op) {
      const bool has = bsh != 0;               // the predecessor op, in the tile (SEG: in this shard)
      const uint64_t k = d.f1 - ri;
      const bool seam_op = !has && tseam && r == ff;   // k_fc_seam's
      if (!seam_op) {
        bool gap;
        if (has) {
          const uint64_t kq = kp - ri;
          if (k <= kq) {                       // an index rewind: the general path's survivor pass
            if (SEG) bad = true;
            else rare |= 2u;
          }
          gap = k > kq && k - kq > 1;
        } else {
          gap = k > 0;
        }
        if (gap) {
          const int gs = st ? st : EWAL_PANIC_INDEX_GAP;
          if (SEG) atomicMin(&sg.sagg[sh].first_fail, ((unsigned long long)r << 8) | (uint32_t)gs);
          else atomicMax(&ds->fc.fail_inv, ~(((unsigned long long)r << 8) | (uint32_t)gs));
        }
      }
      // op k is ents[k] (the shard's region: [fs[s], fs[s + 1]))
      const uint64_t room = SEG ? (uint64_t)(sg.fs[sh + 1] - lo) : a.ecap;
      if (k < room) {
        ewal_entry e;
        e.term = d.f0;
        e.index = d.f1;
        e.data_off = SEG ? d.edoff - sg.soff[sh] : d.edoff;
        e.data_len = d.edlen;
        e.type = d.etype;
        e.data_nil = d.enil;
        if (!(a.ablate & 8)) {
          pe = e;
          pidx = (SEG ? lo : 0u) + k;
          pend = true;
        }
      }
    }
    if (SEG && bad) atomicOr(&sg.sagg[sh].bad, 1u);
  }
  if (pend) {
    if (SEG) a.ents[pidx] = pe;
    else store_entry_nt(a.ents + pidx, pe);
  }
  if (SEG) aflush();
  // flags of every lane, then one atomic per wave
  uint32_t rr = rare;
  for (int o = 32; o; o >>= 1) rr |= (uint32_t)__shfl_xor((int)rr, o);
  if (lane == 0 && rr) atomicOr(&ds->fc.rare, rr);
  if (__ballot(irr) && lane == 0) atomicOr(&ds->irregular, 1u);
}

// After k_fc and the seam pass (one workgroup): does the regular case hold?
// Then ReadAll's metadata rule (wal/wal.go:178-183) over the listed metadata
// frames and the ResultDev gather k_result makes on the general path (the
// few frames it needs re-read in parallel); spec_n = frames, or 0 (the host
// takes the general path); Small -> host-mapped memory.
__device__ void fc_result(const uint8_t *__restrict__ buf, uint64_t B, const uint64_t *__restrict__ cpos, uint64_t ccap,
                          uint64_t ecap, uint64_t ri, const uint32_t *__restrict__ mlist, Small *ds, ResultDev *o,
                          Small *h, uint4 (*s_w)[6], RecDesc *s_d) {
  const uint64_t K = ds->total;
  if (!fc_valid(ds, ccap, ecap)) {
    __syncthreads();
    if (threadIdx.x == 0) {
      ds->spec_n = 0;
      *h = *ds;
    }
    return;
  }
  const uint32_t tid = threadIdx.x;
  const uint64_t fm = ds->fc.meta_inv ? ~ds->fc.meta_inv : ~0ull;
  if (fm != ~0ull && ds->nmeta > 1) {
    const RecDesc m = fc_frame_fields(buf, B, cpos[fm], s_w[tid]);
    for (uint32_t i = tid; i < ds->nmeta; i += blockDim.x) {
      const uint32_t r = mlist[i];
      if (r <= fm) continue;
      const RecDesc d = fc_frame_fields(buf, B, cpos[r], s_w[tid]);
      bool eq = d.dlen == m.dlen;
      for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = buf[d.doff + k] == buf[m.doff + k];
      if (!eq) atomicMax(&ds->fc.fail_inv, ~(((unsigned long long)r << 8) | EWAL_ERR_METADATA_CONFLICT));
    }
  }
  __threadfence();
  __syncthreads();
  // the frames the result needs: first failure, last entry, last state,
  // first metadata, last op -- one thread each
  const unsigned long long key = ds->fc.fail_inv ? ~ds->fc.fail_inv : ~0ull;
  const long long le = (long long)ds->fc.last_entry1 - 1, ls = (long long)ds->fc.last_state1 - 1;
  const long long lo = (long long)ds->lastop - 1;
  const long long want[5] = {key != ~0ull ? (long long)(key >> 8) : -1, le, ls, fm != ~0ull ? (long long)fm : -1, lo};
  if (tid < 5 && want[tid] >= 0) s_d[tid] = fc_frame_fields(buf, B, cpos[want[tid]], s_w[tid]);
  __syncthreads();
  if (tid != 0) return;
  ResultDev res;
  memset(&res, 0, sizeof(res));
  res.agg.first_fail = key != ~0ull ? (key >> 8) : ~0ull;
  res.agg.last_entry = le;
  res.agg.last_state = ls;
  res.agg.first_meta = fm;
  if (key != ~0ull) {
    res.fail = s_d[0];
    res.fail.st = (int32_t)(key & 0xff);
  }
  if (le >= 0) res.lastent = s_d[1];
  if (ls >= 0) res.sd = s_d[2];
  if (fm != ~0ull) res.md = s_d[3];
  res.last.chained = ds->fc.last_chained;
  res.nops = ds->nsel3;
  res.klast = lo >= 0 ? s_d[4].f1 - ri : 0;
  res.errflag = ds->errflag;
  *o = res;
  ds->spec_n = (uint32_t)K;
  *h = *ds;
}

// The index-gap rule (wal/wal.go:173) for each tile's first op whose
// predecessor op lies in an earlier tile: the nearest earlier tile with ops
// holds it (its last op's Index) -- in the same shard when that tile's last
// op lies at or after the shard's first frame.  One thread per tile; the
// edge frames' CRC checks k_fc left to it too, and (single WAL) the fold of
// the tiles' reductions: one atomic per workgroup and quantity.
#define FC_SEAM_SCAN 4096   // tiles scanned back for the predecessor (beyond: the general path)
template <bool SEG>
__global__ __launch_bounds__(256) void k_fc_seam(const uint8_t *__restrict__ buf, uint64_t B,
                                                 const uint64_t *__restrict__ cpos,
                                                 const uint32_t *__restrict__ g_shift,
                                                 const TileRec *__restrict__ trec,
                                                 const ewal_entry *__restrict__ ents, uint64_t ri_one, uint64_t ccap,
                                                 uint64_t ecap, Small *ds, SegArgs sg,
                                                 const uint32_t *__restrict__ mlist, ResultDev *o, Small *h) {
  __shared__ unsigned long long s_fail;
  __shared__ uint32_t s_red[5];   // last entry + 1, last state + 1, ~first meta, last op + 1, ops
  __shared__ uint32_t s_last;
  __shared__ uint4 s_w[SEG ? 1 : 256][6];
  __shared__ RecDesc s_d[SEG ? 1 : 6];
  if (!fc_ran(ds, ccap, ecap)) {   // single WAL: the verdict "general path" to the host
    if (!SEG && blockIdx.x == 0 && threadIdx.x == 0) {
      ds->spec_n = 0;
      *h = *ds;
    }
    return;
  }
  const uint64_t K = ds->total;
  const uint32_t ntiles = (uint32_t)((K + FC_TILE - 1) / FC_TILE);
  // a grid-strided pass over the tiles: the grid (a few workgroups per CU) is
  // sized before the candidate count is known, so every workgroup takes part
  // in the fold below instead of a capacity-sized grid of empty workgroups
  const uint32_t nblocks = gridDim.x;
  if (!SEG) {
    if (threadIdx.x == 0) {
      s_fail = ~0ull;
      s_red[0] = s_red[1] = s_red[3] = s_red[4] = 0;
      s_red[2] = 0;
    }
    __syncthreads();
  }
  unsigned long long fail = ~0ull;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x) {
    const TileRec tr = trec[t];
    const uint32_t r0 = t * FC_TILE;
    const uint32_t rl = min(r0 + FC_TILE, (uint32_t)K) - 1;   // the tile's last frame
    for (int w = 0; w < 2; ++w) {   // the edge frames' CRC checks k_fc left
      const bool first = w == 0;
      if (first ? !tr.dfirst : (!tr.dlast || (tr.dfirst && rl == r0))) continue;
      const uint32_t r = first ? r0 : rl;
      const uint32_t seed = first ? trec[t - 1].lastcrc : tr.seed1;
      const bool next = !first || (tr.dlast && rl == r0);   // P(data end) from the next tile
      const uint32_t pe = next ? trec[t + 1].pfo0 : tr.pe0;
      uint32_t chained;
      const int st = fc_check_one(g_shift, tr.type[w], tr.crc[w], seed, tr.pfd[w], pe, tr.dlen[w], &chained);
      if (st) {
        const unsigned long long key = ((unsigned long long)r << 8) | (uint32_t)st;
        if (SEG) atomicMin(&sg.sagg[shard_of(sg.fs, sg.ns, r)].first_fail, key);
        else fail = min(fail, key);
      }
      if (!SEG && r + 1 == K) ds->fc.last_chained = chained;
    }
    if (tr.seam && tr.count && tr.first_frame < K) {
      const uint32_t f = tr.first_frame;
      uint64_t ri = ri_one;
      uint32_t sh = 0, lo = 0;
      if (SEG) {
        sh = shard_of(sg.fs, sg.ns, f);
        ri = sg.ri[sh];
        lo = sg.fs[sh];
      }
      bool has = false, far = false;
      uint64_t pidx = 0;
      uint32_t scanned = 0;
      for (int64_t u = (int64_t)t - 1; u >= 0 && (uint64_t)(u + 1) * FC_TILE > lo; --u) {
        if (++scanned > FC_SEAM_SCAN) {   // a very long run of tiles without entries: the general path
          far = true;
          break;
        }
        const TileRec q = trec[u];
        if (!q.count) continue;
        has = !SEG || q.last_frame >= lo;
        pidx = q.last_index;
        break;
      }
      if (far) {
        if (SEG) atomicOr(&sg.sagg[sh].bad, 1u);
        else atomicOr(&ds->fc.rare, 8u);
      } else {
        const uint64_t k = tr.first_index - ri;
        bool gap;
        if (has) {
          const uint64_t kq = pidx - ri;
          if (k <= kq) {
            if (SEG) atomicOr(&sg.sagg[sh].bad, 1u);
            else atomicOr(&ds->fc.rare, 2u);
          }
          gap = k > kq && k - kq > 1;
        } else {
          gap = k > 0;
        }
        if (gap) {
          const unsigned long long key = ((unsigned long long)f << 8) | EWAL_PANIC_INDEX_GAP;
          if (SEG) atomicMin(&sg.sagg[sh].first_fail, key);
          else fail = min(fail, key);
        }
      }
    }
    if (!SEG) {
      fail = min(fail, tr.fail);
      if (tr.last_entry1) atomicMax(&s_red[0], tr.last_entry1);
      if (tr.last_state1) atomicMax(&s_red[1], tr.last_state1);
      if (tr.meta1) atomicMax(&s_red[2], ~(tr.meta1 - 1u));
      if (tr.lastop1) atomicMax(&s_red[3], tr.lastop1);
      if (tr.count) atomicAdd(&s_red[4], tr.count);
    }
  }
  if (!SEG) {
    if (fail != ~0ull) atomicMin(&s_fail, fail);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (s_fail != ~0ull) atomicMax(&ds->fc.fail_inv, ~s_fail);
      if (s_red[0]) atomicMax(&ds->fc.last_entry1, s_red[0]);
      if (s_red[1]) atomicMax(&ds->fc.last_state1, s_red[1]);
      if (s_red[2]) atomicMax(&ds->fc.meta_inv, ~(unsigned long long)(uint32_t)~s_red[2]);
      if (s_red[3]) atomicMax(&ds->lastop, s_red[3]);
      if (s_red[4]) atomicAdd(&ds->nsel3, s_red[4]);
      __threadfence();
      s_last = atomicAdd(&ds->fc_done, 1u) == nblocks - 1;
    }
    __syncthreads();
    if (s_last) {   // the last workgroup: every tile's reductions are in
      __threadfence();
      fc_result(buf, B, cpos, ccap, ecap, ri_one, mlist, ds, o, h, s_w, s_d);
    }
  }
}

// ---- batched ReadAll (ewal_readall_batch_device) on the fused pass --------
// fs[s] = first frame at or after the shard's first byte (frame r is
// candidate r on the regular path); the per-shard reductions initialised.
__global__ void k_shard_start_fc(const uint64_t *__restrict__ cpos, uint64_t ccap, const uint64_t *__restrict__ soff,
                                 uint32_t ns, uint32_t *__restrict__ fs, ShardAgg *__restrict__ sagg, Small *ds) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > ns) return;
  const uint64_t K = ds->total;
  const uint32_t n = (uint32_t)(K <= ccap && K < 0xffffff00ull ? K : 0);
  if (s == ns) {
    fs[ns] = n;
    return;
  }
  const uint64_t o = soff[s];
  uint32_t a = 0, b = n;
  while (a < b) {
    const uint32_t m = (a + b) >> 1;
    if (cpos[m] < o) a = m + 1; else b = m;
  }
  fs[s] = a;
  ShardAgg g;
  g.first_fail = ~0ull;
  g.last_entry = -1;
  g.last_state = -1;
  g.first_meta = ~0ull;
  g.ent_first = ~0ull;
  g.lastop = 0;
  g.bad = soff[s + 1] > o && (a >= n || cpos[a] != o);   // the shard does not open on a candidate
  g.term1 = 0;
  g.term_st = 0;
  g.term_off = 0;
  sagg[s] = g;
}

// Per shard: ReadAll's metadata rule (wal/wal.go:178-183) over the metadata
// frames k_fc<true> listed.
__global__ void k_meta_batch_fc(const uint8_t *__restrict__ buf, uint64_t B, const uint64_t *__restrict__ cpos,
                                uint64_t ccap, uint64_t ecap, const uint32_t *__restrict__ mlist, const Small *ds,
                                SegArgs sg) {
  __shared__ uint4 s_w[256][6];
  if (!fc_valid_seg(ds, ccap, ecap)) return;
  const uint32_t nm = ds->nmeta;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nm; i += gridDim.x * blockDim.x) {
    const uint32_t r = mlist[i];
    const uint32_t s = shard_of(sg.fs, sg.ns, r);
    const unsigned long long fm = sg.sagg[s].first_meta;
    if (fm == ~0ull || r <= fm) continue;
    const RecDesc d = fc_frame_fields(buf, B, cpos[r], s_w[threadIdx.x]);
    const RecDesc m = fc_frame_fields(buf, B, cpos[fm], s_w[threadIdx.x]);
    bool eq = d.dlen == m.dlen;
    for (uint64_t k = 0; eq && k < d.dlen; ++k) eq = buf[d.doff + k] == buf[m.doff + k];
    if (!eq) atomicMin(&sg.sagg[s].first_fail, ((unsigned long long)r << 8) | EWAL_ERR_METADATA_CONFLICT);
  }
}

// Per shard: its ReadAll result (k_result_batch's assembly with first_fail =
// frame << 8 | status), the frames it needs re-read from the stream -- eight
// lanes per shard, one frame each (first failure, last entry, last frame,
// first metadata, last state, last op), lane 0 assembles.
__global__ __launch_bounds__(256) void k_result_batch_fc(const uint8_t *__restrict__ buf, uint64_t B,
                                                         const uint64_t *__restrict__ cpos, uint64_t ccap,
                                                         uint64_t ecap, const Small *ds, SegArgs sg,
                                                         ewal_result *__restrict__ out,
                                                         unsigned long long *__restrict__ ent_first) {
  __shared__ uint4 s_w[256][6];
  __shared__ RecDesc s_d[256];
  const uint32_t s = (blockIdx.x * blockDim.x + threadIdx.x) >> 3, k = threadIdx.x & 7;
  if (!fc_valid_seg(ds, ccap, ecap)) return;   // (a void pass: the host discards out[])
  const bool in = s < sg.ns;
  ShardAgg A;
  uint32_t f0 = 0, f1 = 0;
  if (in) {
    A = sg.sagg[s];
    f0 = sg.fs[s];
    f1 = A.term1 ? A.term1 - 1u : sg.fs[s + 1];   // the shard's frames end at its terminal (a torn tail)
    long long fr = -1;
    switch (k) {
    case 0: fr = A.first_fail != ~0ull ? (long long)(A.first_fail >> 8) : -1; break;
    case 1: fr = A.last_entry; break;
    case 2: fr = f1 > f0 ? (long long)f1 - 1 : -1; break;
    case 3: fr = A.first_meta != ~0ull ? (long long)A.first_meta : -1; break;
    case 4: fr = A.last_state; break;
    case 5: fr = A.lastop ? (long long)A.lastop - 1 : -1; break;
    default: break;
    }
    if (fr >= 0) s_d[threadIdx.x] = fc_frame_fields(buf, B, cpos[fr], s_w[threadIdx.x]);
  }
  __syncthreads();
  if (!in || k != 0) return;
  const RecDesc *D = s_d + threadIdx.x;   // D[k]: lane k's frame
  const uint64_t so = sg.soff[s], ri = sg.ri[s];
  ewal_result o;
  memset(&o, 0, sizeof(o));
  o.fail_record = -1;
  o.fail_offset = -1;
  o.metadata_off = -1;
  o.n_records = (int64_t)(f1 - f0);
  o.n_candidates = (int64_t)(sg.fs[s + 1] - f0);
  o.n_runs = 1;
  unsigned long long ef = 0;
  if (A.first_fail != ~0ull) {
    const uint32_t fr = (uint32_t)(A.first_fail >> 8);
    o.status = (int32_t)(A.first_fail & 0xff);
    o.fail_record = (int64_t)(fr - f0);
    o.fail_offset = (int64_t)(D[0].off - so);
    o.n_records = o.fail_record;
    if (o.status == EWAL_ERR_UNEXPECTED_TYPE) o.detail = D[0].type;
    if (o.status == EWAL_PANIC_INDEX_GAP) o.detail = (int64_t)D[0].f1;
  } else if (A.term1 && A.term_st != EWAL_OK) {   // ReadAll returns decoder.decode's error (wal/wal.go:197-201)
    o.status = A.term_st;
    o.fail_record = (int64_t)(f1 - f0);
    o.fail_offset = (int64_t)(A.term_off - so);
  } else {
    const uint64_t enti = A.last_entry >= 0 ? D[1].f1 : 0;
    o.enti = enti;
    if (enti < ri) {
      o.status = EWAL_ERR_INDEX_NOT_FOUND;
    } else if (f1 > f0) {
      // the running CRC after the shard's last frame: the stored CRC of a
      // verified frame (crcType re-seeds to it; every other frame's check
      // passed, so computed == stored)
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
      o.n_ents = A.lastop ? (int64_t)(D[5].f1 - ri + 1) : 0;
      ef = o.n_ents ? f0 : 0;   // op k of the shard is bents[fs[s] + k]
    }
  }
  if (A.bad) o.flags = EW_SHARD_BAD;   // replayed alone by the host (its fields here are void)
  out[s] = o;
  ent_first[s] = ef;
}

// The batch's verdict on the fused pass (one thread): the pass ran over every
// candidate -> spec_n = frames (shards it could not decide carry EW_SHARD_BAD
// in their result), else 0; Small -> host-mapped memory.
__global__ void k_batch_gate_fc(Small *ds, uint64_t ccap, uint64_t ecap, uint64_t B, Small *h) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t K = ds->total;
  const bool ok = fc_valid_seg(ds, ccap, ecap);
  ds->spec_n = ok ? (uint32_t)K : 0u;
  *h = *ds;
}
