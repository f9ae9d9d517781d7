// ewal_api.hip -- C ABI + host driver for the device pipeline (single TU).
//
// Implements include/ewal.h's compute entry points.  The pipeline for
// (*WAL).ReadAll (wal/wal.go:164-216) is:
//   k_stream (one HBM pass) -> unit scan -> k_frame (speculative framing +
//   decode; fallback: k_link, runs, pointer jumping, k_decode) -> k_check ->
//   k_result (k_check also places the entry ops; rare: k_gap, k_ents)
// and the host only classifies the chain's terminal frame and assembles the
// ewal_result from a few device reductions.  No CPU decoding or CRC happens
// on this path; without a GPU every call returns EWAL_E_NODEVICE.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <vector>

#include "crc_math.h"
#include "wal_kernels.hip"
#include "aux_kernels.hip"
#include "msg_kernels.hip"
#include "frame_fields.hip"
#include "frame_kernels.hip"
#include "ewal_stage.h"

#define EW_CHECK(x)                                                          \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::fprintf(stderr, "ewal: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return EWAL_E_HIP;                                                     \
    }                                                                        \
  } while (0)

namespace {

struct DevTables {
  uint32_t *slice = nullptr;  // [16][256] slicing-by-16 (the first 4 tables: slicing-by-4)
  uint32_t *shift = nullptr;  // [48][4][256]
  uint32_t *unib = nullptr;   // [16][8][16] nibble tables of S_{256 (15 - m)}, m = 0..15 (k_stream's unit lins)
};

// Grow-only device buffer owned by a ctx (freed by its destructor when the
// ctx is deleted; ewal_ctx_destroy makes the ctx's device current first).
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  // take o's allocation (ours is released first)
  void adopt(DevBuf &o) {
    release();
    p = o.p;
    cap = o.cap;
    o.p = nullptr;
    o.cap = 0;
  }
  // grow-only device buffer
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  template <typename T> T *as() { return static_cast<T *>(p); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Grow-only pinned host buffer mapped into the device address space: small
// per-call tables the kernels read and write in place (no DMA copies to queue
// behind a caller's bulk transfers).
struct HostBuf {
  void *h = nullptr, *d = nullptr;
  size_t cap = 0;
  HostBuf() = default;
  HostBuf(const HostBuf &) = delete;
  HostBuf &operator=(const HostBuf &) = delete;
  ~HostBuf() { release(); }
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    const size_t want = std::max<size_t>(n, 4096);
    hipError_t e = hipHostMalloc(&h, want, hipHostMallocMapped);
    if (e != hipSuccess) { h = nullptr; return e; }
    e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) { release(); return e; }
    cap = want;
    return hipSuccess;
  }
  template <typename T> T *host() { return static_cast<T *>(h); }
  template <typename T> T *dev() { return static_cast<T *>(d); }
  void release() {
    if (h) (void)hipHostFree(h);
    h = d = nullptr;
    cap = 0;
  }
};

}  // namespace

struct ewal_ctx {
  int device = 0;
  int num_cu = 256;
  int ablate = 0;      // EWAL_STREAM_ABLATE (timing experiments only; results are wrong)
  int frame_wg = 3;    // k_frame resident workgroups per CU (EWAL_FRAME_WG: A/B timing)
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evs0 = nullptr, evs1 = nullptr;
  hipEvent_t evf0 = nullptr, evf1 = nullptr;   // around k_frames (the serial pipeline)
  hipEvent_t evf_start = nullptr;              // the frame pass's start: evf0, or evs1 when nothing ran between
  bool frames_timed = false;                   // evf0 / evf1 bracket this call's frame pass
  bool spin = true;                            // ew_sync: spin on the stream instead of blocking (profiles/r05/
                                               // host_gap_*.txt: the call's host time 21 -> 14 us on configs[0])
  // record-dense WALs: the stream pass also stores vh[] (every super-piece's
  // first 128-B half) and the frame pass takes its prefixes at 128-B
  // granularity.  vh_opt: 0 auto (the ctx's previous single ReadAll had >= 4
  // frames per 4 KiB unit: dense_hint), 1 on, -1 off (EWAL_OPT_VH_ON / _OFF)
  int vh_opt = 0;
  bool dense_hint = false;
  // the batched ReadAll's own hint: its previous batch had >= EW_VH_BATCH_FPU
  // frames per 4 KiB unit (configs[2]-shaped shards: 3.5)
  bool dense_hint_batch = false;
  uint32_t *vh_next = nullptr;                 // run_stream: the vh[] of this call's stream pass
  DevBuf vhb;
  std::map<uint32_t, DevTables> tables;
  std::map<uint32_t, std::unique_ptr<ewal::CrcTables>> host_tables;
  DevBuf encw, encs, lbstat, gagg, slow, mlist, pf, v, pwave, ux, tagg, tpx, wcnt, slots, cbase, ovf, cpos, clen, nxt, exc, E, rs, jl, vis, entry, on, rec_cand, rd, opf, ops, kk, kkrev, suf,
      ents, recs, tmp, small, sdesc, snaps, hbuf_dev, xpos, walk, fpos, ulist, uitems, uarena, ftrec, fpl, fucb,
      fnfp, frbase, fsp, ftcb, fown, fcl, ftl, ftcnt;
  DevBuf rents, rmlist, rulist;   // materialise_records' k_check outputs (never the ReadAll's own ents)
  HostBuf hsdesc;                  // esnap_verify_packed's per-file table (host-mapped)
  // esnap_verify_packed's residual decode (esnap_copy_field): the batch's
  // buffer, per file its residual slot (-1: none), per slot its segments
  const uint8_t *snap_buf = nullptr;
  uint32_t snap_n = 0;
  std::vector<int32_t> snap_rmap;
  std::vector<uint64_t> snap_rfirst, snap_rcnt;
  DevBuf sgather, ssegs, srlist, sgoff, srcnt, srfirst;
  std::vector<ewal_unrec> unrec;   // XXX_unrecognized of the last ReadAll's result (side list)
  uint64_t unrec_bytes = 0;
  // the side arena of split byte fields (Record.Data / Entry.Data repeated
  // with several non-empty segments): the general path gathers their
  // concatenations here (ewal_copy_split_bytes)
  DevBuf cat;
  uint64_t cat_bytes = 0;
  bool cat_retry = false;
  bool defer_first = false;   // ewal_readall_range_device: frame 0's CRC check is the caller's
  bool last_deferred = false;
  std::vector<std::vector<uint8_t>> bsplit_bytes;   // per shard replayed alone: its split bytes
  // batched ReadAll (ewal_readall_batch_device): shard tables, results, ents
  DevBuf bfs, bsoff, bri, bsagg, bres, bef, bents, bshard, hmask;
  // batched raftpb.Message decode (emsg_decode_batch_device)
  DevBuf moff, mlen, mcnt, mfirst, mout, ments, mscnt, msfirst, msegs;
  uint64_t mtotal = 0, mstotal = 0;
  std::vector<uint64_t> bent_first, bnents;   // per shard: first ent in bents, count
  std::vector<std::vector<ewal_unrec>> bunrec;       // per shard replayed alone: its XXX_unrecognized side list
  std::vector<std::vector<uint8_t>> bunrec_bytes;
  Small *h_small = nullptr;        // host-mapped pinned mirrors (written by k_export_small / k_result)
  ResultDev *h_res = nullptr;
  Small *h_small_dev = nullptr;    // their device-side addresses
  ResultDev *h_res_dev = nullptr;
  // results of the last readall
  uint64_t last_n = 0, last_nents = 0;
  uint64_t last_k = 0;     // candidates of the previous call (sizes k_frame's descriptors)
  uint32_t epoch = 0;      // k_check look-back epoch (24 bits)
  int fused = 1;           // the fused frame + check pass first (EWAL_FUSED=0: the general path only)
  bool rd_valid = false;   // c->rd holds the last call's per-frame descriptors
  bool rec_valid = false;     // the last ReadAll's last_n frames can be described (ewal_copy_records,
                              // ewal_range_info)
  bool rec_rebuild = false;   // the last ReadAll was decided by the fused pass and the stream pass's
                              // state (cpos, pwave, v) is still its own: ewal_copy_records can rebuild
                              // the descriptors from it and the caller's stream bytes
  // the last ReadAll's frame pass when it decided the call (rec_rebuild):
  // ewal_copy_range_info reads its reductions instead of rebuilding descriptors
  bool fi_valid = false;
  int fi_tsh = 0;
  FrArgs fi_a{};
  Small fi_small{};
  DevBuf rfr;                // RangeFr
  const uint8_t *last_buf = nullptr;   // the last ReadAll's stream (materialise_records)
  uint64_t last_B = 0, last_ri = 0;
  uint64_t pfcap = 0;      // pf = [P at data starts | P at frame starts], pfcap each
  bool last_ok = false;
  bool scan_valid = false;   // cpos / pwave / cbase hold the current stream pass's candidates and prefixes
  bool fr_rew_hint = false;  // the last single ReadAll needed the frame pass's rewind mode
  // the batched ReadAll's: the shards of the ctx's previous batch (same shard
  // count and bytes) whose indexes went back run the next batch's frame pass in
  // rewind mode (k_shard_hint) instead of a second pass over their tiles
  std::vector<uint32_t> brew_hint;
  uint32_t brew_ns = 0;
  uint64_t brew_B = 0;
  uint32_t brew_clcap = 1u << 20;
  DevBuf fhint;
  uint64_t last_q = 0;       // where the last ReadAll's frame chain ended (decoder.decode's terminal)
  // the overlapped pipeline (single WAL): two streams on disjoint CU masks --
  // the stream pass's chunks on ov_s[0] (ov_cu[0] CUs), the frame pass's on
  // ov_s[1] (ov_cu[1] CUs) -- and the events that order them
  hipStream_t ov_s[2] = {nullptr, nullptr};
  bool ov_opt = false;       // EWAL_OPT_OVERLAP
  int ov_state = 0;          // 0 not tried, 1 ready, -1 unavailable (the serial pipeline)
  int ov_chunks = 4, ov_fcus = 32, ov_cu[2] = {0, 0};
  int ov_nofr = 0;           // tools/ hooks builds only (EWAL_OV_NOFR): every frame chunk after the stream pass
  std::vector<hipEvent_t> ov_ev;
  DevBuf fticks;             // per chunk: its frame pass's tile counter
  StreamArgs ov_sa{};        // the call's stream-pass arguments (run_stream), launched per chunk
};

// The HBM staging buffer of host bytes (ewal_readall_host, ewal_stage_*):
// refilling or reallocating it takes away the stream the last ReadAll's
// descriptors are rebuilt from when that ReadAll read it.
static hipError_t stage_ensure(ewal_ctx *c, size_t n) {
  if (c->last_buf && c->last_buf == c->hbuf_dev.as<uint8_t>()) {
    c->rec_rebuild = false;
    c->last_buf = nullptr;
  }
  return c->hbuf_dev.ensure(n);
}

static int get_tables(ewal_ctx *c, uint32_t poly, DevTables **out) {
  auto it = c->tables.find(poly);
  if (it != c->tables.end()) {
    *out = &it->second;
    return 0;
  }
  auto ht = std::make_unique<ewal::CrcTables>(poly);
  DevTables t;
  EW_CHECK(hipMalloc(&t.slice, sizeof(ht->slice16)));
  EW_CHECK(hipMalloc(&t.shift, ht->shift.size() * sizeof(uint32_t)));
  EW_CHECK(hipMemcpy(t.slice, ht->slice16, sizeof(ht->slice16), hipMemcpyHostToDevice));
  EW_CHECK(hipMemcpy(t.shift, ht->shift.data(), ht->shift.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  {   // unib[m][k][d] = S_{256 (15 - m)}(d << 4k): the shift of super-piece m's lin to its unit's end
    std::vector<uint32_t> un(16 * 128);
    auto apply = [&](int lvl, uint32_t x) {
      const uint32_t *tb = &ht->shift[(size_t)lvl * 1024];
      return tb[x & 0xff] ^ tb[256 + ((x >> 8) & 0xff)] ^ tb[512 + ((x >> 16) & 0xff)] ^ tb[768 + (x >> 24)];
    };
    for (int m = 0; m < 16; ++m)
      for (int k = 0; k < 8; ++k)
        for (uint32_t d = 0; d < 16; ++d) {
          uint32_t x = d << (4 * k);
          const uint32_t n = 256u * (15u - (uint32_t)m);
          for (int lvl = 0; lvl < 32; ++lvl)
            if ((n >> lvl) & 1u) x = apply(lvl, x);
          un[(size_t)m * 128 + k * 16 + d] = x;
        }
    EW_CHECK(hipMalloc(&t.unib, un.size() * sizeof(uint32_t)));
    EW_CHECK(hipMemcpy(t.unib, un.data(), un.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  c->host_tables[poly] = std::move(ht);
  c->tables[poly] = t;
  *out = &c->tables[poly];
  return 0;
}

// diagnostics of the batch path's decisions (tools/ builds only: the product
// build reads no environment variable)
static inline bool ew_debug() {
#ifdef EW_ABLATION_HOOKS
  return std::getenv("EWAL_DEBUG") != nullptr;
#else
  return false;
#endif
}

static inline unsigned grid_for(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// hipcub DeviceSelect::Flagged(counting 0.., flags) -> out, count in *d_count
static int select_flagged(ewal_ctx *c, const uint8_t *flags, uint32_t n, uint32_t *out, uint32_t *d_count) {
  hipcub::CountingInputIterator<uint32_t> it(0);
  size_t bytes = 0;
  EW_CHECK(hipcub::DeviceSelect::Flagged(nullptr, bytes, it, flags, out, d_count, (int)n, c->stream));
  EW_CHECK(c->tmp.ensure(bytes));
  EW_CHECK(hipcub::DeviceSelect::Flagged(c->tmp.p, bytes, it, flags, out, d_count, (int)n, c->stream));
  return 0;
}

// The general framing path's per-candidate arrays (lengths, links, link
// exceptions): allocated only when that path runs, so the regular path's
// first call does not pay for them.
static int ensure_cand_aux(ewal_ctx *c, uint64_t ccap) {
  EW_CHECK(c->clen.ensure(ccap * 8));
  EW_CHECK(c->nxt.ensure(ccap * 4));
  EW_CHECK(c->exc.ensure(ccap));
  return 0;
}

// The overflow path of the candidate compaction (the list outgrew ccap):
// slots -> dense list again (k_compact), then the overflow units (k_rescan).
static int compact_cands(ewal_ctx *c, const uint8_t *d_buf, uint64_t B, uint32_t nunits, uint64_t ccap) {
  if (int rc = ensure_cand_aux(c, ccap)) return rc;
  Small *ds = c->small.as<Small>();
  EW_CHECK(hipMemsetAsync(&ds->novf, 0, 4, c->stream));
  hipLaunchKernelGGL(k_compact, dim3(grid_for(nunits, 256)), dim3(256), 0, c->stream, d_buf, nunits,
                     c->wcnt.as<uint32_t>(), c->cbase.as<unsigned long long>(), c->slots.as<uint16_t>(),
                     c->cpos.as<uint64_t>(), c->clen.as<uint64_t>(), ccap, c->ovf.as<uint32_t>(), &ds->novf);
  hipLaunchKernelGGL(k_rescan, dim3(64), dim3(256), 0, c->stream, d_buf, B, c->ovf.as<uint32_t>(), &ds->novf,
                     c->cbase.as<unsigned long long>(), c->cpos.as<uint64_t>(), c->clen.as<uint64_t>(), ccap);
  EW_CHECK(hipGetLastError());
  return 0;
}

// The candidates of the units with more than EW_SLOTS of them (small
// records) into cpos (k_rescan: each such unit scanned again, its candidates
// written from its base); Small.novf cleared, so a pass over the candidate
// list can run again.
static int rescan_overflow(ewal_ctx *c, const uint8_t *d_buf, uint64_t B, uint64_t ccap) {
  if (int rc = ensure_cand_aux(c, ccap)) return rc;
  Small *ds = c->small.as<Small>();
  hipLaunchKernelGGL(k_rescan, dim3(64), dim3(256), 0, c->stream, d_buf, B, c->ovf.as<uint32_t>(), &ds->novf,
                     c->cbase.as<unsigned long long>(), c->cpos.as<uint64_t>(), c->clen.as<uint64_t>(), ccap);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipMemsetAsync(&ds->novf, 0, 4, c->stream));
  return 0;
}

// Capacity of the dense candidate list for a B-byte stream: a frame is at
// least 12 bytes, but candidates denser than one per 128 B only come from
// tiny records; those calls grow the list (compact_cands) and run again.
static inline uint64_t cand_cap(uint64_t B) { return std::min<uint64_t>(B / 128 + 65536, 0xfffffff0ull); }

// Run the HBM pass (k_stream) and the unit scan over d_buf[0..B): fills
// c->v, c->pwave; with find_cand also the dense, position-sorted candidate
// list cpos[] (k_uapply's epilogue; units with more than EW_SLOTS candidates
// are counted in Small.novf and filled in by k_rescan later), its size in
// Small.total.  Asynchronous: nothing waits for the device here.
// The stream pass's and unit scan's workspace for a B-byte stream.
static int stream_ensure(ewal_ctx *c, uint64_t B, int find_cand) {
  const uint64_t nunits64 = B / EW_WAVE_BYTES + 1;
  if (nunits64 >= 0xffff0000ull) return EWAL_E_INVAL;
  const uint32_t nunits = (uint32_t)nunits64;
  const uint32_t nstiles = (nunits + EW_TILE_UNITS - 1) / EW_TILE_UNITS;
  EW_CHECK(c->v.ensure((size_t)nunits * EW_VPU * 4));
  EW_CHECK(c->pwave.ensure((size_t)nunits * 4));
  EW_CHECK(c->wcnt.ensure((size_t)nunits * 4));
  EW_CHECK(c->cbase.ensure((size_t)nunits * 8));
  if (find_cand) {
    EW_CHECK(c->slots.ensure((size_t)nunits * EW_SLOTS * 2));
    EW_CHECK(c->ovf.ensure((size_t)nunits * 4));
    if (EW_SPLIT_CAND) EW_CHECK(c->hmask.ensure((size_t)nunits * 16));   // {flagged pieces, of them: group 3}
  }
  EW_CHECK(c->ux.ensure((size_t)nunits * 4));
  EW_CHECK(c->tagg.ensure((size_t)nstiles * 16));
  EW_CHECK(c->tpx.ensure((size_t)nstiles * 16));
  EW_CHECK(c->gagg.ensure((size_t)((nstiles + 1023) / 1024) * 16));
  return 0;
}

// The per-frame descriptors of the last ReadAll live in (or are rebuilt from)
// ctx state that any other pipeline call overwrites: forget them.
static void forget_records(ewal_ctx *c) {
  c->rec_valid = false;
  c->rd_valid = false;
  c->rec_rebuild = false;
  c->last_n = 0;
}

static int run_cand_scan(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, int find_cand, uint64_t ccap);

// The HBM pass (k_stream) over d_buf[0..B): v[] and, with find_cand, the
// flagged pieces (hmask).  With scan also the candidate tests and the unit
// scan (run_cand_scan): P at every unit start (pwave) and, with find_cand,
// the dense, position-sorted candidate list cpos[] (units with more than
// EW_SLOTS candidates are counted in Small.novf and filled in by k_rescan
// later), its size in Small.total.  Asynchronous: nothing waits here.
static int run_stream(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, int find_cand, uint64_t ccap,
                      bool scan = true, bool launch = true) {
  forget_records(c);   // cpos / pwave / v are about to change (readall_impl sets them again after)
  c->scan_valid = false;
  const uint64_t nunits64 = B / EW_WAVE_BYTES + 1;
  if (nunits64 >= 0xffff0000ull) return EWAL_E_INVAL;
  const uint32_t nunits = (uint32_t)nunits64;
  if (int rc = stream_ensure(c, B, find_cand)) return rc;
  Small *ds = c->small.as<Small>();   // zeroed by k_stream (workgroup 0), the first kernel of every call
  StreamArgs a;
  a.buf = d_buf;
  a.B = B;
  a.nunits = nunits;
  a.find_cand = find_cand;
  a.ablate = c->ablate;
  a.g_slice = tb->slice;
  a.g_shift = tb->shift;
  a.v = c->v.as<uint32_t>();
  a.wcnt = c->wcnt.as<uint32_t>();
  a.slots = find_cand ? c->slots.as<uint16_t>() : nullptr;
  a.hmask = find_cand && EW_SPLIT_CAND ? c->hmask.as<unsigned long long>() : nullptr;
  a.small = ds;
  a.u_begin = 0;
  a.u_end = nunits;
  a.vh = find_cand ? c->vh_next : nullptr;
  c->vh_next = nullptr;
  a.ulin = c->ux.as<uint32_t>();   // (find_cand, EW_ULIN: the unit lins, read by the frame pass's phase A)
  a.g_unib = tb->unib;
  c->ov_sa = a;
  if (!launch) return 0;   // the overlapped pipeline launches the stream pass in chunks (frames_pass)
  unsigned grid = (unsigned)std::min<uint64_t>((nunits + 2 * EW_WAVES - 1) / (2 * EW_WAVES), (uint64_t)c->num_cu);
#ifdef EW_ABLATION_HOOKS
  if (const char *e = std::getenv("EWAL_STREAM_CUS")) grid = std::min<unsigned>(grid, (unsigned)std::atoi(e));   // tools/ only
#endif
  EW_CHECK(hipEventRecord(c->evs0, c->stream));
  if (find_cand)
    hipLaunchKernelGGL(k_stream<true>, dim3(grid), dim3(EW_THREADS), 0, c->stream, a);
  else
    hipLaunchKernelGGL(k_stream<false>, dim3(grid), dim3(EW_THREADS), 0, c->stream, a);
  EW_CHECK(hipGetLastError());
#ifdef EW_ABLATION_HOOKS
  if (!std::getenv("EWAL_NO_MID_EVENTS"))   // tools/ only
#endif
    EW_CHECK(hipEventRecord(c->evs1, c->stream));
  if (!scan) return 0;
  return run_cand_scan(c, tb, d_buf, B, find_cand, ccap);
}

// The general path's inputs from the stream pass's v[] / hmask: the exact
// candidate tests (k_cand -> slots, wcnt), the unit scan (pwave, cbase) and
// the dense candidate list (cpos).  The fused frame pass needs none of them;
// they run when the general path or the descriptors (ewal_copy_records) do.
static int run_cand_scan(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, int find_cand, uint64_t ccap) {
  const uint32_t nunits = (uint32_t)(B / EW_WAVE_BYTES + 1);
  const uint32_t nstiles = (nunits + EW_TILE_UNITS - 1) / EW_TILE_UNITS;
  Small *ds = c->small.as<Small>();
  if (find_cand && EW_SPLIT_CAND && !(EW_XS & 8))   // the exact tests on the flagged pieces -> slots, wcnt
  {
    EW_CHECK(c->cpos.ensure(ccap * 8));
    // four groups of 64 units per wave while that still gives every CU 16
    // waves (fewer, longer waves starve the CUs on small streams)
    const bool g4 = (uint64_t)nunits >= (uint64_t)std::max(1, c->num_cu) * 16 * 64 * 4;
    if (g4)
      hipLaunchKernelGGL(k_cand<4>, dim3(grid_for(nunits, 64 * EW_CAND_WAVES * 4)), dim3(64 * EW_CAND_WAVES), 0,
                         c->stream, d_buf, B, nunits, c->hmask.as<unsigned long long>(), c->slots.as<uint16_t>(),
                         c->wcnt.as<uint32_t>());
    else
      hipLaunchKernelGGL(k_cand<1>, dim3(grid_for(nunits, 64 * EW_CAND_WAVES)), dim3(64 * EW_CAND_WAVES), 0,
                         c->stream, d_buf, B, nunits, c->hmask.as<unsigned long long>(), c->slots.as<uint16_t>(),
                         c->wcnt.as<uint32_t>());
  }
  ScanArgs s;
  s.nunits = nunits;
  s.ntiles = nstiles;
  s.v = c->v.as<uint32_t>();
  s.wcnt = c->wcnt.as<uint32_t>();
  s.g_shift = tb->shift;
  s.pwave = c->pwave.as<uint32_t>();
  s.cbase = c->cbase.as<unsigned long long>();
  s.ux = c->ux.as<uint32_t>();
  s.tagg = c->tagg.as<uint32_t>();
  s.tcnt = s.tagg + nstiles;
  s.tpx = c->tpx.as<uint32_t>();
  s.tcb = (unsigned long long *)(c->tpx.as<uint8_t>() + (size_t)nstiles * 8);
  s.gcnt = c->gagg.as<unsigned long long>();
  s.gagg = (uint32_t *)(s.gcnt + (nstiles + 1023) / 1024);
  s.total = &ds->total;
  s.slots = find_cand ? c->slots.as<uint16_t>() : nullptr;
  s.cpos = find_cand ? c->cpos.as<uint64_t>() : nullptr;
  s.ccap = ccap;
  s.ovf = find_cand ? c->ovf.as<uint32_t>() : nullptr;
  s.novf = &ds->novf;
  // one wave per 1 MiB tile: k_uagg one 16-wave workgroup per CU (its S_256
  // table fills the LDS), k_uapply likewise (one staging of its tables per CU)
  const unsigned agrid = std::min<uint32_t>((nstiles + 15) / 16, (uint32_t)c->num_cu);
  const unsigned sgrid = std::min<uint32_t>((nstiles + 15) / 16, (uint32_t)c->num_cu);
  hipLaunchKernelGGL(k_uagg, dim3(agrid), dim3(1024), 0, c->stream, s);
  const uint32_t ngroups = (nstiles + 1023) / 1024;
  if (ngroups > 1024) return EWAL_E_INVAL;   // k_tfix: at most 1024 tile groups (1 TiB)
  hipLaunchKernelGGL(k_tscan, dim3(ngroups), dim3(1024), 0, c->stream, s);
  hipLaunchKernelGGL(k_tfix, dim3(ngroups), dim3(1024), 0, c->stream, s, ngroups);
  hipLaunchKernelGGL(k_uapply, dim3(sgrid), dim3(1024), 0, c->stream, s);
  EW_CHECK(hipGetLastError());
  c->scan_valid = find_cand != 0;
  // units with more than EW_SLOTS candidates (ds->novf) are left out of cpos
  // here: k_frame then declines to speculate and the host runs k_rescan
  return 0;
}

static int sync_small(ewal_ctx *c) {
  hipLaunchKernelGGL(k_export_small, dim3(1), dim3(64), 0, c->stream, c->small.as<Small>(), c->h_small_dev);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipStreamSynchronize(c->stream));
  if (c->h_small->errflag) return EWAL_E_TIMEOUT;
  return 0;
}

// decoder.decode at frame start q when q is not a candidate of the chain
// (wal/decoder.go:28-39 + io.ReadFull's EOF/ErrUnexpectedEOF rule); L is the
// int64 at q (valid when q + 8 <= B).  EWAL_FRAME_FITS: a whole frame lies
// at q that the candidate filter did not admit -- k_walk decodes it.
#define EWAL_FRAME_FITS (-100)
static int classify_terminal(uint64_t B, uint64_t q, int64_t L) {
  if (q == B) return EWAL_OK;
  if (B - q < 8) return EWAL_ERR_UNEXPECTED_EOF;
  const uint64_t rem = B - q - 8;
  if (L < 0) return EWAL_PANIC_NEG_LENGTH;
  if ((uint64_t)L > rem) return rem == 0 ? EWAL_OK : EWAL_ERR_UNEXPECTED_EOF;
  return EWAL_FRAME_FITS;
}

// Pointer jumping over runs of consecutive candidates (the candidate links
// from k_link's nxt / exc): run ends E, jump levels J, marks cleared.
struct JumpState {
  uint32_t R = 0;
  int top = 0;
  bool ready = false;
};
static int jump_prepare(ewal_ctx *c, uint64_t K, JumpState *js) {
  Small *ds = c->small.as<Small>();
  const uint32_t K32 = (uint32_t)K;
  EW_CHECK(c->E.ensure((size_t)K * 4));
  int rc = select_flagged(c, c->exc.as<uint8_t>(), K32, c->E.as<uint32_t>(), &ds->nsel);
  if (rc) return rc;
  if ((rc = sync_small(c))) return rc;
  const uint32_t R = c->h_small->nsel;
  int top = 0;
  while ((1ull << top) < R) ++top;
  EW_CHECK(c->jl.ensure((size_t)R * 4 * (top + 1)));
  EW_CHECK(c->vis.ensure(R));
  EW_CHECK(c->entry.ensure((size_t)R * 4));
  uint32_t *J = c->jl.as<uint32_t>();
  hipLaunchKernelGGL(k_runs, dim3(grid_for(R, 256)), dim3(256), 0, c->stream, c->E.as<uint32_t>(), R,
                     c->nxt.as<uint32_t>(), J);
  for (int k = 1; k <= top; ++k)
    hipLaunchKernelGGL(k_jump, dim3(grid_for(R, 256)), dim3(256), 0, c->stream, J + (size_t)(k - 1) * R,
                       J + (size_t)k * R, R);
  EW_CHECK(hipMemsetAsync(c->vis.p, 0, R, c->stream));
  EW_CHECK(hipMemsetAsync(c->entry.p, 0xff, (size_t)R * 4, c->stream));
  EW_CHECK(hipGetLastError());
  js->R = R;
  js->top = top;
  js->ready = true;
  return 0;
}

// Marks the chain segment starting at candidate `cand` (segments are marked
// in position order); returns its terminal candidate and the offset after it.
static int jump_mark(ewal_ctx *c, const JumpState &js, uint32_t cand, uint32_t *last_cand, uint64_t *q_out) {
  Small *ds = c->small.as<Small>();
  const uint32_t R = js.R;
  uint32_t *J = c->jl.as<uint32_t>();
  hipLaunchKernelGGL(k_jstart, dim3(1), dim3(64), 0, c->stream, c->E.as<uint32_t>(), R, cand, c->vis.as<uint8_t>(),
                     c->entry.as<uint32_t>(), &ds->ci);
  for (int k = js.top; k >= 0; --k)
    hipLaunchKernelGGL(k_mark, dim3(grid_for(R, 256)), dim3(256), 0, c->stream, J + (size_t)k * R,
                       c->vis.as<uint8_t>(), R);
  hipLaunchKernelGGL(k_entry, dim3(grid_for(R, 256)), dim3(256), 0, c->stream, c->E.as<uint32_t>(),
                     c->nxt.as<uint32_t>(), J, c->vis.as<uint8_t>(), R, c->entry.as<uint32_t>(), &ds->ci);
  EW_CHECK(hipGetLastError());
  int rc = sync_small(c);
  if (rc) return rc;
  const uint32_t lc = c->h_small->ci.last_cand;
  uint64_t pl[2];
  EW_CHECK(hipMemcpyAsync(&pl[0], c->cpos.as<uint64_t>() + lc, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&pl[1], c->clen.as<uint64_t>() + lc, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  *last_cand = lc;
  *q_out = pl[0] + 8 + pl[1];
  return 0;
}

// The marked candidates -> rec_cand (ascending); returns their count.
static int jump_finish(ewal_ctx *c, uint64_t K, const JumpState &js, uint64_t *n_out) {
  Small *ds = c->small.as<Small>();
  const uint32_t K32 = (uint32_t)K;
  EW_CHECK(c->on.ensure(K));
  EW_CHECK(c->rec_cand.ensure((size_t)K * 4));
  hipLaunchKernelGGL(k_member, dim3(grid_for(K, 256)), dim3(256), 0, c->stream, c->E.as<uint32_t>(), js.R,
                     c->vis.as<uint8_t>(), c->entry.as<uint32_t>(), K32, c->on.as<uint8_t>());
  int rc = select_flagged(c, c->on.as<uint8_t>(), K32, c->rec_cand.as<uint32_t>(), &ds->nsel2);
  if (rc) return rc;
  if ((rc = sync_small(c))) return rc;
  *n_out = c->h_small->nsel2;
  return 0;
}

// Framing when the candidates do not form one chain from byte 0: the chain
// from candidate 0 by pointer jumping; returns its length n (c->rec_cand),
// its last candidate and its terminal q.
static int frame_irregular(ewal_ctx *c, uint64_t K, ewal_result *out, JumpState *js, uint64_t *n_out,
                           uint32_t *last_cand, uint64_t *q_out) {
  int rc = jump_prepare(c, K, js);
  if (rc) return rc;
  out->n_runs = js->R;
  if ((rc = jump_mark(c, *js, 0, last_cand, q_out))) return rc;
  return jump_finish(c, K, *js, n_out);
}

static int read_le64_at(ewal_ctx *c, const uint8_t *d_buf, uint64_t B, uint64_t q, int64_t *L) {
  *L = 0;
  if (q + 8 > B) return 0;
  EW_CHECK(hipMemcpyAsync(L, d_buf + q, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  return 0;
}

// The chain's terminal q holds a frame the candidate filter did not admit
// (classify_terminal == EWAL_FRAME_FITS): k_walk decodes frames from q on
// until the chain meets a candidate again (marked from there by pointer
// jumping; the walk continues at that segment's terminal), ends, or a frame
// fails.  The walked frames are appended to `xs` (ascending); *tst is the
// final terminal class (EWAL_OK when a walked frame fails: k_check reports
// that frame), *q_out its offset.  `regular`: every candidate is on the
// chain already (no segment can follow).  On return *n_cands is the number
// of chain candidates (rec_cand when js->ready, else candidates 0..n-1).
static int walk_chain(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, uint64_t K, bool regular,
                      JumpState *js, uint32_t pc, uint64_t *n_cands, uint64_t *q_out, int *tst,
                      std::vector<uint64_t> &xs) {
  const uint32_t xcap = 1u << 16;
  EW_CHECK(c->xpos.ensure((size_t)xcap * 8));
  EW_CHECK(c->walk.ensure(sizeof(WalkOut)));
  uint64_t q = *q_out;
  bool has_seed = false;
  uint32_t seed = 0;
  bool marked = false;   // a segment after the first was marked: rec_cand needs rebuilding
  for (;;) {
    hipLaunchKernelGGL(k_walk, dim3(1), dim3(64), 0, c->stream, d_buf, B, q, c->cpos.as<uint64_t>(), K, pc,
                       (int)has_seed, seed, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift,
                       c->xpos.as<uint64_t>(), xcap, c->walk.as<WalkOut>());
    EW_CHECK(hipGetLastError());
    WalkOut w;
    EW_CHECK(hipMemcpyAsync(&w, c->walk.p, sizeof(w), hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
    if (w.n) {
      const size_t at = xs.size();
      xs.resize(at + w.n);
      EW_CHECK(hipMemcpy(xs.data() + at, c->xpos.p, (size_t)w.n * 8, hipMemcpyDeviceToHost));
    }
    if (w.stopped) {   // a walked frame fails: ReadAll ends there
      *tst = EWAL_OK;
      *q_out = w.x;
      break;
    }
    if (w.term >= 0) {
      *tst = w.term;
      *q_out = w.x;
      break;
    }
    if (w.resume == ~0ull) {   // the list filled: continue from x
      q = w.x;
      has_seed = true;
      seed = w.seed;
      continue;
    }
    // the chain meets candidate w.resume: mark the segment from there
    if (regular) return EWAL_E_INVAL;   // impossible: every candidate lies before q
    if (!js->ready) {
      int rc = jump_prepare(c, K, js);
      if (rc) return rc;
    }
    uint32_t lc = 0;
    int rc = jump_mark(c, *js, (uint32_t)w.resume, &lc, &q);
    if (rc) return rc;
    marked = true;
    int64_t qlen = 0;
    if ((rc = read_le64_at(c, d_buf, B, q, &qlen))) return rc;
    const int t = classify_terminal(B, q, qlen);
    if (t != EWAL_FRAME_FITS) {
      *tst = t;
      *q_out = q;
      break;
    }
    pc = lc;
    has_seed = false;
  }
  if (marked) return jump_finish(c, K, *js, n_cands);
  return 0;
}

// The frame pass (k_frames + k_frames_seam, frame_kernels.hip) over the
// stream pass's v[] / hmask: ONE host sync.  *done when the regular case held
// (ResultDev in c->h_res, ents in c->ents); otherwise the caller runs the
// general path over the same stream pass.  ents and the metadata list grow
// and the pass reruns (once) when it reported them too small.
#ifndef EW_SEAM_WGS
#define EW_SEAM_WGS 2
#endif
// log2 of the units per tile: the largest of 256 (1 MiB tiles), 64 and 16
// that still gives every wave of the grid two tiles (more, smaller tiles on
// small streams keep the waves busy; large tiles amortise the per-tile work)
static int fr_tsh(const ewal_ctx *c, uint32_t nunits) {
#ifdef EW_ABLATION_HOOKS
  if (const char *e = std::getenv("EWAL_TSH")) {   // tools/ timing builds only: an instantiated tile size
    const int t = std::atoi(e);
    return t >= 8 ? 8 : t >= 6 ? 6 : 4;
  }
#endif
  const uint64_t w2 = (uint64_t)FR_WAVES * std::max(1, c->num_cu) * 2;
  return (uint64_t)nunits >= 256 * w2 ? 8 : (uint64_t)nunits >= 64 * w2 ? 6 : 4;
}
// the frame pass's workgroups (one per CU; tools/ hooks builds: EWAL_FRAME_CUS)
static int fr_cus(const ewal_ctx *c) {
#ifdef EW_ABLATION_HOOKS
  if (const char *e = std::getenv("EWAL_FRAME_CUS")) return std::max(1, std::atoi(e));   // tools/ only
#endif
  return std::max(1, c->num_cu);
}
static void fr_launch_result_batch(ewal_ctx *c, int tsh, const FrArgs &a, const FrSeg &sg) {
  const dim3 g(grid_for((uint64_t)sg.ns * 64, 256));
  if (tsh == 8)
    hipLaunchKernelGGL(k_result_batch_fr<8>, g, dim3(256), 0, c->stream, a, sg, c->bres.as<ewal_result>(),
                       c->bef.as<unsigned long long>());
  else if (tsh == 6)
    hipLaunchKernelGGL(k_result_batch_fr<6>, g, dim3(256), 0, c->stream, a, sg, c->bres.as<ewal_result>(),
                       c->bef.as<unsigned long long>());
  else
    hipLaunchKernelGGL(k_result_batch_fr<4>, g, dim3(256), 0, c->stream, a, sg, c->bres.as<ewal_result>(),
                       c->bef.as<unsigned long long>());
}
static int fr_ensure(ewal_ctx *c, uint32_t nunits, uint32_t ntiles) {
  EW_CHECK(c->ftrec.ensure((size_t)ntiles * sizeof(FrTile)));
  EW_CHECK(c->ftcnt.ensure((size_t)ntiles * 4));
  EW_CHECK(c->fpl.ensure((size_t)nunits * 4));
  EW_CHECK(c->fucb.ensure((size_t)nunits * 4));
  return 0;
}
static FrArgs fr_args(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, uint32_t nunits, uint32_t ntiles,
                      uint64_t ri, ewal_entry *ents, uint64_t ecap, uint32_t mcap) {
  FrArgs a;
  a.buf = d_buf;
  a.B = B;
  a.nunits = nunits;
  a.ntiles = ntiles;
  a.hmask = (const ulonglong2 *)c->hmask.p;
  a.v = c->v.as<uint32_t>();
  a.g_slice = tb->slice;
  a.g_shift = tb->shift;
  a.pl = c->fpl.as<uint32_t>();
  a.ucb = c->fucb.as<uint32_t>();
  a.trec = c->ftrec.as<FrTile>();
  a.tcnt = c->ftcnt.as<uint32_t>();
  a.ents = ents;
  a.ecap = ecap;
  a.mlist = c->mlist.as<uint64_t>();
  a.mcap = mcap;
  a.ri = ri;
  a.ds = c->small.as<Small>();
  a.rew = 0;
  a.own = nullptr;
  a.clist = nullptr;
  a.ccap = 0;
  a.tlist = nullptr;
  a.ntl = 0;
  a.t0 = 0;
  a.nrun = 0;
  a.tick = nullptr;
  a.vh = nullptr;
  a.ulin = c->ux.as<uint32_t>();
  return a;
}
// the call's scratch as k_stream leaves it (a rerun of the frame pass, or the
// general path after it)
static int reset_small(ewal_ctx *c) {
  Small *ds = c->small.as<Small>();
  EW_CHECK(hipMemsetAsync(ds, 0, sizeof(Small), c->stream));
  if (c->defer_first) EW_CHECK(hipMemsetAsync(&ds->defer_first, 1, 1, c->stream));
  return 0;
}
// The call's device times from its events (ev1 already synchronised):
// device_ms ev0 -> ev1, stream_ms evs0 -> evs1, post_ms evs1 -> ev1 and, when
// the frame pass ran as one launch, frames_ms evf0 -> evf1.
#ifndef EW_FR_EVF0
#define EW_FR_EVF0 0
#endif
// The call's wait for its last kernel: a spin on the stream's completion
// (c->spin) instead of the runtime's blocking wait, whose wake-up sits between
// the device finishing and the host seeing the result.
// Only on the ctx's own stream: a caller-owned stream (ewal_ctx_set_stream,
// e.g. torch's) may hold the caller's other work, which a spin would wait
// out on a whole host core; there the runtime's blocking wait is used.
static hipError_t ew_sync(ewal_ctx *c) {
  bool spin = c->spin && c->own_stream;
#ifdef EW_ABLATION_HOOKS
  if (const char *e = std::getenv("EWAL_SPIN")) spin = std::atoi(e) != 0;   // tools/ only
#endif
  if (!spin) return hipStreamSynchronize(c->stream);
  hipError_t e;
  while ((e = hipStreamQuery(c->stream)) == hipErrorNotReady) {
  }
  return e;
}
static int set_times(ewal_ctx *c, ewal_result *o, uint32_t n = 1) {
  float dev = 0, str = 0, post = 0, fr = 0;
  EW_CHECK(hipEventElapsedTime(&dev, c->ev0, c->ev1));
#ifdef EW_ABLATION_HOOKS
  if (std::getenv("EWAL_NO_MID_EVENTS")) {   // tools/ only: the whole call's time alone
    for (uint32_t i = 0; i < n; ++i) o[i].device_ms = dev;
    return 0;
  }
#endif
  EW_CHECK(hipEventElapsedTime(&str, c->evs0, c->evs1));
  EW_CHECK(hipEventElapsedTime(&post, c->evs1, c->ev1));
  if (c->frames_timed) EW_CHECK(hipEventElapsedTime(&fr, c->evf_start ? c->evf_start : c->evf0, c->evf1));
  for (uint32_t i = 0; i < n; ++i) {
    o[i].device_ms = dev;
    o[i].stream_ms = str;
    o[i].post_ms = post;
    o[i].frames_ms = fr;
  }
  return 0;
}

// ---- the overlapped pipeline (round 5) ----------------------------------------
// Both passes are issue-bound on the SIMDs rather than HBM-bound: k_stream
// keeps 98 % of its speed on 224 of the 256 CUs (1.675 vs 1.638 ms over
// 8 GiB) but loses 11 % on 192, and the frame pass over 8 GiB takes 0.345 ms
// on 256 CUs, 0.51 on 128 and 0.89 on 64 (profiles/r05/cu_sweep.txt).  So the
// post-stream pass is hidden by giving it a few CUs for the whole call: the
// stream pass runs in chunks (whole tiles) on a stream whose CU mask holds
// ov_cu[0] CUs, and the frame pass of chunk k runs on a second stream masked
// to the other ov_cu[1] CUs as soon as chunk k's stream pass is done (an
// event); the last chunk's frame pass takes the whole chip on the call's own
// stream, then the seam pass.  A tile's frame pass reads only its own units'
// v[] / hmask (frames reaching into the next tile go to the seam pass), so a
// chunk needs nothing of the chunks after it.
// A ctx whose masked streams are still alive when the process exits
// (ewal_ctx_destroy never called) used to crash in __cxa_finalize: the HIP
// runtime's own teardown destroyed the CU-masked streams after the profiler /
// runtime state they depend on was gone (profiles/r05: tools/ov_child.py under
// rocprofv3, SIGSEGV at exit after four correct calls).  The library now keeps
// the ctxs that own such streams and destroys those streams from an atexit
// handler registered when the first one is created -- after the HIP runtime's
// initialisation, so it runs before the runtime's own teardown.  Callers should
// still destroy every ctx before exit (include/ewal.h); this covers the ones
// that do not (a Go process that exits with a live ctx).
static std::mutex &ov_reg_mu() {
  static std::mutex *m = new std::mutex();   // never destroyed: used from the atexit handler
  return *m;
}
static std::set<ewal_ctx *> &ov_reg() {
  static std::set<ewal_ctx *> *r = new std::set<ewal_ctx *>();
  return *r;
}
static void ov_release_streams(ewal_ctx *c) {
  for (hipStream_t &st : c->ov_s)
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
      st = nullptr;
    }
}
static void ov_atexit() {
  std::lock_guard<std::mutex> g(ov_reg_mu());
  for (ewal_ctx *c : ov_reg()) {
    (void)hipSetDevice(c->device);
    ov_release_streams(c);
    c->ov_state = -1;
  }
  ov_reg().clear();
}
static void ov_register(ewal_ctx *c) {
  static std::once_flag once;
  std::call_once(once, [] { std::atexit(ov_atexit); });
  std::lock_guard<std::mutex> g(ov_reg_mu());
  ov_reg().insert(c);
}
static void ov_unregister(ewal_ctx *c) {
  std::lock_guard<std::mutex> g(ov_reg_mu());
  ov_reg().erase(c);
}
static bool ov_ready(ewal_ctx *c) {
  if (c->ov_state) return c->ov_state > 0;
  c->ov_state = -1;
  const int n = std::max(2, c->num_cu);
  const int nf = std::max(1, std::min(c->ov_fcus, n / 2));
  std::vector<uint32_t> ms((n + 31) / 32, 0u), mf((n + 31) / 32, 0u);
  for (int i = 0; i < n; ++i) (i < n - nf ? ms : mf)[i >> 5] |= 1u << (i & 31);
  if (hipExtStreamCreateWithCUMask(&c->ov_s[0], (uint32_t)ms.size(), ms.data()) != hipSuccess) {
    c->ov_s[0] = nullptr;
    return false;
  }
  if (hipExtStreamCreateWithCUMask(&c->ov_s[1], (uint32_t)mf.size(), mf.data()) != hipSuccess) {
    (void)hipStreamDestroy(c->ov_s[0]);
    c->ov_s[0] = c->ov_s[1] = nullptr;
    return false;
  }
  c->ov_cu[0] = n - nf;
  c->ov_cu[1] = nf;
  c->ov_state = 1;
  ov_register(c);
  return true;
}
static hipError_t ov_events(ewal_ctx *c, size_t n) {
  while (c->ov_ev.size() < n) {
    hipEvent_t e;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) return r;
    c->ov_ev.push_back(e);
  }
  return hipSuccess;
}
// the stream pass over units [ub, ue) on stream st with at most cus workgroups
static void ov_stream_chunk(ewal_ctx *c, uint32_t ub, uint32_t ue, int cus, hipStream_t st) {
  StreamArgs a = c->ov_sa;
  a.u_begin = ub;
  a.u_end = ue;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((ue - ub + 2 * EW_WAVES - 1) / (2 * EW_WAVES),
                                                                         (uint64_t)cus));
  hipLaunchKernelGGL(k_stream<true>, dim3(grid), dim3(EW_THREADS), 0, st, a);
}
template <bool SEG>
static void fr_launch_frames(int tsh, uint32_t nt, const FrArgs &a, const FrSeg &sg, int cus, hipStream_t st) {
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(grid_for(nt, FR_WAVES), (uint64_t)cus));
  if (a.vh) {   // record-dense: the 128-B prefixes
    if (tsh == 8) hipLaunchKernelGGL((k_frames<SEG, 8, true>), dim3(grid), dim3(FR_THREADS), 0, st, a, sg);
    else if (tsh == 6) hipLaunchKernelGGL((k_frames<SEG, 6, true>), dim3(grid), dim3(FR_THREADS), 0, st, a, sg);
    else hipLaunchKernelGGL((k_frames<SEG, 4, true>), dim3(grid), dim3(FR_THREADS), 0, st, a, sg);
    return;
  }
  if (tsh == 8) hipLaunchKernelGGL((k_frames<SEG, 8>), dim3(grid), dim3(FR_THREADS), 0, st, a, sg);
  else if (tsh == 6) hipLaunchKernelGGL((k_frames<SEG, 6>), dim3(grid), dim3(FR_THREADS), 0, st, a, sg);
  else hipLaunchKernelGGL((k_frames<SEG, 4>), dim3(grid), dim3(FR_THREADS), 0, st, a, sg);
}
template <bool SEG>
static void fr_launch_seam(ewal_ctx *c, int tsh, uint32_t nt, const FrArgs &a, const FrSeg &sg, ResultDev *o,
                           Small *h) {
  const unsigned sgrid = (unsigned)std::min<uint64_t>(grid_for(nt, 256), (uint64_t)std::max(1, c->num_cu) * EW_SEAM_WGS);
  if (tsh == 8) hipLaunchKernelGGL((k_frames_seam<SEG, 8>), dim3(sgrid), dim3(256), 0, c->stream, a, sg, o, h);
  else if (tsh == 6) hipLaunchKernelGGL((k_frames_seam<SEG, 6>), dim3(sgrid), dim3(256), 0, c->stream, a, sg, o, h);
  else hipLaunchKernelGGL((k_frames_seam<SEG, 4>), dim3(sgrid), dim3(256), 0, c->stream, a, sg, o, h);
}
// The stream pass and the frame pass of a single WAL, overlapped (above).
// Replaces run_stream's launch + the first fr_launch; the events evs0 / evs1
// bracket the stream chunks (stream_ms), ev1 is recorded by the caller.
static int ov_launch(ewal_ctx *c, int tsh, uint32_t nunits, uint32_t ntiles, const FrArgs &a0) {
  const uint32_t tu = 1u << tsh;
  const uint32_t C = (uint32_t)std::max(1, std::min<int>(c->ov_chunks, (int)ntiles));
  const uint32_t tpc = (ntiles + C - 1) / C;
  hipStream_t sA = c->ov_s[0], sB = c->ov_s[1];
  EW_CHECK(ov_events(c, 2 * (size_t)C + 2));
  hipEvent_t *ev = c->ov_ev.data();   // [0] fork, [1 + k] stream chunk k, [1 + C + k] frames chunk k
  EW_CHECK(c->fticks.ensure((size_t)C * 4));
  EW_CHECK(hipMemsetAsync(c->fticks.p, 0, (size_t)C * 4, c->stream));
  EW_CHECK(hipEventRecord(ev[0], c->stream));   // fork: both streams after the call's work so far
  EW_CHECK(hipStreamWaitEvent(sA, ev[0], 0));
  EW_CHECK(hipStreamWaitEvent(sB, ev[0], 0));
  EW_CHECK(hipEventRecord(c->evs0, sA));
  Small *ds = c->small.as<Small>();
  for (uint32_t k = 0; k < C; ++k) {
    const uint32_t tb = k * tpc, te = std::min(ntiles, tb + tpc);
    if (tb >= te) break;
    const uint32_t ub = tb * tu, ue = std::min(nunits, te * tu);
    ov_stream_chunk(c, ub, ue, c->ov_cu[0], sA);
    EW_CHECK(hipEventRecord(ev[1 + k], sA));
    const bool last = te == ntiles || c->ov_nofr;
    hipStream_t sf = last ? c->stream : sB;   // the last chunk's frames: the whole chip, on the call's stream
    EW_CHECK(hipStreamWaitEvent(sf, ev[1 + k], 0));
    if (k == 0 && c->defer_first) EW_CHECK(hipMemsetAsync(&ds->defer_first, 1, 1, sf));   // (after k_stream zeroed Small)
    FrArgs a = a0;
    a.t0 = tb;
    a.nrun = te - tb;
    a.tick = c->fticks.as<uint32_t>() + k;
    fr_launch_frames<false>(tsh, te - tb, a, FrSeg{}, last ? std::max(1, c->num_cu) : c->ov_cu[1], sf);
    if (!last) EW_CHECK(hipEventRecord(ev[1 + C + k], sB));
    if (te == ntiles) {
      EW_CHECK(hipEventRecord(c->evs1, sA));
      if (k && !c->ov_nofr) EW_CHECK(hipStreamWaitEvent(c->stream, ev[C + k], 0));   // join: the frames before
      break;
    }
  }
  EW_CHECK(hipGetLastError());
  fr_launch_seam<false>(c, tsh, ntiles, a0, FrSeg{}, c->h_res_dev, c->h_small_dev);
  EW_CHECK(hipGetLastError());
  return 0;
}

static int frames_pass(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, uint64_t ri, uint64_t ecap,
                       bool *done, bool ov = false) {
  *done = false;
  const uint32_t nunits = (uint32_t)(B / EW_WAVE_BYTES + 1);
  const int tsh = fr_tsh(c, nunits);
  const uint32_t tu = 1u << tsh, ntiles = (nunits + tu - 1) / tu;
  if (int rc = fr_ensure(c, nunits, ntiles)) return rc;
  uint32_t mcap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(c->mlist.cap / 8, 4096), 0xffffffffull);
  // rewind mode: entry indexes go back (wal/wal.go:173 truncates ents).  A
  // ctx whose last ReadAll met rewinds starts in it (a restarted member
  // replays the same WAL again and again); a call that then meets none
  // clears the hint.
  bool rew = c->fr_rew_hint;
  uint32_t clcap = 0;
  for (int pass = 0; pass < 4; ++pass) {
    EW_CHECK(c->ents.ensure((size_t)ecap * sizeof(ewal_entry)));
    EW_CHECK(c->mlist.ensure((size_t)mcap * 8));
    if (pass) if (int rc = reset_small(c)) return rc;
    FrArgs a = fr_args(c, tb, d_buf, B, nunits, ntiles, ri, c->ents.as<ewal_entry>(), ecap, mcap);
    a.vh = c->ov_sa.vh;   // the stream pass's vh[] when it stored one (record-dense WALs)
    if (rew) {
      clcap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(clcap, ecap), 0xffffffffull);
      EW_CHECK(c->fown.ensure((size_t)ecap * 8));
      EW_CHECK(c->fcl.ensure((size_t)clcap * 4));
      EW_CHECK(hipMemsetAsync(c->fown.p, 0, (size_t)ecap * 8, c->stream));
      a.rew = 1;
      a.own = c->fown.as<unsigned long long>();
      a.clist = c->fcl.as<uint32_t>();
      a.ccap = clcap;
    }
    if (ov && pass == 0) {
      if (int rc = ov_launch(c, tsh, nunits, ntiles, a)) return rc;
      c->frames_timed = false;
    } else {
      // the stream pass's end event doubles as the frame pass's start on the
      // first pass (no work between them): one marker fewer between the two
      // kernels (EW_FR_EVF0=1: its own event, A/B)
      if (EW_FR_EVF0 || pass) {
        EW_CHECK(hipEventRecord(c->evf0, c->stream));
        c->evf_start = c->evf0;
      } else {
        c->evf_start = c->evs1;
      }
#ifdef EW_ABLATION_HOOKS
      const bool mid = !std::getenv("EWAL_NO_MID_EVENTS");   // tools/ only: the markers' own cost
#else
      const bool mid = true;
#endif
      fr_launch_frames<false>(tsh, ntiles, a, FrSeg{}, fr_cus(c), c->stream);
      if (mid) EW_CHECK(hipEventRecord(c->evf1, c->stream));
      fr_launch_seam<false>(c, tsh, ntiles, a, FrSeg{}, c->h_res_dev, c->h_small_dev);
      c->frames_timed = true;
    }
    if (rew)   // the slots more than one op claimed: their last op's entry
      hipLaunchKernelGGL(k_ents_fix, dim3((unsigned)std::max(1, c->num_cu) * 2), dim3(256), 0, c->stream, d_buf, B,
                         (const unsigned long long *)a.own, (const uint32_t *)a.clist, a.ccap, (const Small *)a.ds,
                         a.ents, (const uint64_t *)nullptr, 0u);
    EW_CHECK(hipGetLastError());
    // the call's end event rides behind the last kernel: when the regular
    // case held, the sync below is the call's only wait for the device
    EW_CHECK(hipEventRecord(c->ev1, c->stream));
    EW_CHECK(ew_sync(c));
    const Small *hs = c->h_small;
    if (ew_debug())
      std::fprintf(stderr, "ewal frames: pass %d tsh %d spec %u rare %u irr %u need %llu nmeta %u K %llu\n", pass, tsh,
                   hs->spec_n, hs->fc.rare, hs->irregular, (unsigned long long)hs->fr_need, hs->nmeta,
                   (unsigned long long)hs->total);
    if (hs->errflag) return EWAL_E_TIMEOUT;
    if (hs->spec_n) {
      *done = true;
      c->fr_rew_hint = rew && hs->fr_rews;
      c->fi_valid = true;
      c->fi_tsh = tsh;
      c->fi_a = a;
      c->fi_small = *hs;
      return 0;
    }
    // declined for capacity or rewinds only: room for what it asked / the rewind mode, once more
    const uint32_t rare = hs->fc.rare;
    if (hs->irregular || (rare & ~(2u | 4u | 8u | 64u))) break;
    bool again = false;
    if ((rare & 2u) && !rew) {
      rew = true;
      again = true;
    }
    if (rare & 64u) {
      clcap = hs->fr_ncl + hs->fr_ncl / 8 + 1024;
      again = true;
    }
    if ((rare & 4u) && hs->fr_need > ecap && hs->fr_need < 0xffffff00ull) {
      ecap = hs->fr_need + hs->fr_need / 8 + 1024;
      again = true;
    }
    if ((rare & 8u) && hs->nmeta > mcap) {
      mcap = hs->nmeta + hs->nmeta / 8 + 1024;
      again = true;
    }
    if (!again) break;
  }
  return 0;
}

// XXX_unrecognized of the returned ents / HardState (wal/wal.go:164-216
// returns them inside the structs; raft.pb.go:270 appends each unknown
// field): the entry ops k_check listed that survive in ents (op j is ents[j]
// when the ops' indexes rise by one; after index rewinds, ents[k_j] iff every
// later op has a larger k) and the last HardState.  Their bytes are gathered
// on the device into the side buffer (rare: etcd's encoder never writes
// unknown fields).
static int gather_unrec(ewal_ctx *c, const uint8_t *d_buf, const ResultDev &res, const ReadAllAgg &agg,
                        uint64_t nents) {
  std::vector<UnrecItem> items;
  if (agg.last_state >= 0 && res.sd.pad1) items.push_back(UnrecItem{(uint32_t)agg.last_state, 0, -1, 0, 0});
  if (res.nunrec) {
    std::vector<uint2> ul(res.nunrec);
    EW_CHECK(hipMemcpy(ul.data(), c->ulist.p, (size_t)res.nunrec * sizeof(uint2), hipMemcpyDeviceToHost));
    for (const uint2 &u : ul) {
      int64_t slot = u.y;
      if (res.nonmono) {   // kk = each op's k, kkrev = suffix minimum of kk (the rewind pass above)
        uint64_t k = 0, later = ~0ull;
        EW_CHECK(hipMemcpy(&k, c->kk.as<uint64_t>() + u.y, 8, hipMemcpyDeviceToHost));
        if (u.y + 1 < res.nops)
          EW_CHECK(hipMemcpy(&later, c->kkrev.as<uint64_t>() + u.y + 1, 8, hipMemcpyDeviceToHost));
        if (!(k < later && k < nents)) continue;   // overwritten by a later op
        slot = (int64_t)k;
      }
      items.push_back(UnrecItem{u.x, 0, slot, 0, 0});
    }
  }
  std::sort(items.begin(), items.end(), [](const UnrecItem &a, const UnrecItem &b) { return a.ent < b.ent; });
  const uint32_t m = (uint32_t)items.size();
  if (!m) return 0;
  EW_CHECK(c->uitems.ensure((size_t)m * sizeof(UnrecItem)));
  EW_CHECK(hipMemcpyAsync(c->uitems.p, items.data(), (size_t)m * sizeof(UnrecItem), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_unrec<0>, dim3(grid_for(m, 64)), dim3(64), 0, c->stream, d_buf, c->rd.as<RecDesc>(),
                     c->uitems.as<UnrecItem>(), m, (uint8_t *)nullptr, (const uint8_t *)c->cat.as<uint8_t>());
  EW_CHECK(hipMemcpyAsync(items.data(), c->uitems.p, (size_t)m * sizeof(UnrecItem), hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  uint64_t tot = 0;
  for (UnrecItem &it : items) {
    it.off = tot;
    tot += it.len;
  }
  EW_CHECK(c->uarena.ensure(tot + 16));
  EW_CHECK(hipMemcpyAsync(c->uitems.p, items.data(), (size_t)m * sizeof(UnrecItem), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_unrec<1>, dim3(grid_for(m, 64)), dim3(64), 0, c->stream, d_buf, c->rd.as<RecDesc>(),
                     c->uitems.as<UnrecItem>(), m, c->uarena.as<uint8_t>(), (const uint8_t *)c->cat.as<uint8_t>());
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipStreamSynchronize(c->stream));
  for (const UnrecItem &it : items) c->unrec.push_back(ewal_unrec{it.ent, it.off, it.len});
  c->unrec_bytes = tot;
  return 0;
}

// (*WAL).ReadAll, wal/wal.go:164-216.  Regular case: ONE host sync in all
// (k_check / k_result queued behind k_frame, gated on the device by
// k_spec_gate); the slow framing paths add their own.
static int readall_impl(ewal_ctx *c, const uint8_t *d_buf, uint64_t B, uint64_t ri, ewal_result *out) {
  bool ev1_final = false;   // c->ev1 already recorded behind the call's last kernel (the fused pass)
  std::memset(out, 0, sizeof(*out));
  out->fail_record = -1;
  out->fail_offset = -1;
  out->metadata_off = -1;
  c->last_ok = false;
  c->last_n = 0;
  c->last_nents = 0;
  c->unrec.clear();
  c->unrec_bytes = 0;
  c->cat_bytes = 0;
  c->rd_valid = false;
  c->fi_valid = false;
  c->last_deferred = c->defer_first;
  c->last_buf = d_buf;
  c->last_B = B;
  c->last_ri = ri;
  if (((uintptr_t)d_buf & 15) != 0 && B) return EWAL_E_INVAL;
  DevTables *tb;
  int rc = get_tables(c, 0x82F63B78u, &tb);
  if (rc) return rc;
  EW_CHECK(c->small.ensure(sizeof(Small)));
  EW_CHECK(c->cat.ensure((size_t)1 << 20));   // the split-field side arena (grown on demand, below)
  EW_CHECK(hipEventRecord(c->ev0, c->stream));
  Small *ds = c->small.as<Small>();

  uint64_t n = 0;          // frames on the chain
  uint64_t q = 0;          // terminal frame offset
  uint64_t K = 0;
  int64_t qlen = 0;
  bool regular = false;
  bool decoded = false;    // k_frame's speculative decode holds
  bool spec_checked = false;   // ... and k_check / k_result already ran behind it
  bool fused_done_final = false;   // the fused pass decided the call (its result carries the stored CRCs)
  if (B > 0) {
    uint64_t ccap = cand_cap(B);
    EW_CHECK(c->cpos.ensure(ccap * 8));
    // descriptor capacity of the speculative frame pass: the previous call's
    // frame count with headroom, at least one frame per 4 KiB
    uint64_t rdcap = std::min<uint64_t>(ccap, std::max<uint64_t>(c->last_k + c->last_k / 8 + 1024,
                                                                 B / 4096 + 1024));
    // the overlapped pipeline for large single WALs (ov_launch): the stream
    // pass is launched in chunks by frames_pass
    const uint32_t nunits_ov = (uint32_t)(B / EW_WAVE_BYTES + 1);
    const bool ov = !EW_XS && c->ov_opt && c->fused && B >= (512ull << 20) && fr_tsh(c, nunits_ov) == 8 &&
                    ov_ready(c);
    // record-dense WALs (the ctx's previous ReadAll: >= 4 frames per 4 KiB
    // unit, or EWAL_OPT_VH_ON): the stream pass also stores vh[] and the
    // frame pass takes its prefixes from 128-B boundaries
    const bool vh = c->fused && (c->vh_opt > 0 || (c->vh_opt == 0 && c->dense_hint));
    if (vh) {
      EW_CHECK(c->vhb.ensure(((size_t)B / EW_WAVE_BYTES + 1) * EW_VPU * 4));
      c->vh_next = c->vhb.as<uint32_t>();
    }
    rc = run_stream(c, tb, d_buf, B, 1, ccap, !c->fused, !ov);
    if (rc) return rc;
    if (c->defer_first && !ov) EW_CHECK(hipMemsetAsync(&ds->defer_first, 1, 1, c->stream));   // (Small is zeroed by k_stream)
#if EW_XS
    // timing-only ablation builds: the stream pass alone
    EW_CHECK(hipEventRecord(c->ev1, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
    float xs_ms = 0;
    EW_CHECK(hipEventElapsedTime(&xs_ms, c->ev0, c->ev1));
    out->device_ms = xs_ms;
    EW_CHECK(hipEventElapsedTime(&xs_ms, c->evs0, c->evs1));
    out->stream_ms = xs_ms;
    return 0;
#endif
    bool fused_done = false;
    if (c->fused) {
      const uint64_t ecap = std::max<uint64_t>(rdcap, c->ents.cap / sizeof(ewal_entry));
      rc = frames_pass(c, tb, d_buf, B, ri, ecap, &fused_done, ov);
      if (rc) return rc;
      ev1_final = fused_done;   // ev1 is behind the last kernel unless more work is queued below
      if (!fused_done) {   // the general path over the same stream pass: its candidates and prefixes first
        if ((rc = reset_small(c))) return rc;
        if ((rc = run_cand_scan(c, tb, d_buf, B, 1, ccap))) return rc;
      }
    }
    uint32_t *pf = nullptr;
    bool rescanned = false;
    for (int pass = 0; pass < 3 && !fused_done; ++pass) {
      EW_CHECK(c->rd.ensure(rdcap * sizeof(RecDesc)));
      EW_CHECK(c->pf.ensure(rdcap * 8));
      EW_CHECK(c->slow.ensure(rdcap * 4));
      c->pfcap = rdcap;
      pf = c->pf.as<uint32_t>();
      const unsigned fgrid = (unsigned)std::max(1, c->num_cu) * c->frame_wg;   // persistent: resident WGs per CU
      hipLaunchKernelGGL(k_frame, dim3(fgrid), dim3(256), 0, c->stream, d_buf, B, c->cpos.as<uint64_t>(), ccap,
                         rdcap, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift,
                         c->rd.as<RecDesc>(), pf, pf + rdcap, c->slow.as<uint32_t>(), ds, c->ablate);
      EW_CHECK(hipGetLastError());
      if (pass == 0) {
        // Queue the check behind the frame pass before the host has seen its
        // verdict: k_spec_gate decides on the device (spec_n = frames, or 0)
        // and k_check / k_result run only when it held -- ONE host sync for
        // the whole call in the regular case.
        hipLaunchKernelGGL(k_spec_gate, dim3(1), dim3(64), 0, c->stream, ds, ccap, rdcap, c->h_small_dev);
        hipLaunchKernelGGL(k_decode_slow, dim3(64), dim3(256), 0, c->stream, d_buf, B, c->cpos.as<uint64_t>(),
                           (const uint32_t *)nullptr, c->slow.as<uint32_t>(), ds, c->pwave.as<uint32_t>(),
                           c->v.as<uint32_t>(), tb->slice, tb->shift, c->rd.as<RecDesc>(), pf, pf + rdcap, 0u,
                           c->cat.as<uint8_t>(), (uint64_t)c->cat.cap);
        const uint32_t nbs = grid_for(rdcap, 1024);
        const size_t had = c->lbstat.cap;
        EW_CHECK(c->lbstat.ensure((size_t)nbs * 8));
        c->epoch = (c->epoch + 1) & 0xffffffu;
        if (c->lbstat.cap != had || c->epoch == 0) {
          EW_CHECK(hipMemsetAsync(c->lbstat.p, 0, c->lbstat.cap, c->stream));
          if (c->epoch == 0) c->epoch = 1;
        }
        EW_CHECK(c->opf.ensure((size_t)nbs * 4));
        EW_CHECK(c->mlist.ensure((size_t)rdcap * 4));
        EW_CHECK(c->ents.ensure((size_t)rdcap * sizeof(ewal_entry)));
        EW_CHECK(c->ulist.ensure((size_t)rdcap * sizeof(uint2)));
        SegArgs useg{};
        useg.ulist = c->ulist.as<uint2>();
        hipLaunchKernelGGL(k_check<false>, dim3(nbs), dim3(1024), 0, c->stream, tb->shift, c->rd.as<RecDesc>(),
                           (uint32_t)rdcap, (const uint32_t *)pf, (const uint32_t *)(pf + rdcap), ri,
                           c->lbstat.as<unsigned long long>(), c->epoch, c->opf.as<uint32_t>(),
                           c->ents.as<ewal_entry>(), c->mlist.as<uint32_t>(), ds, useg,
                           (const uint32_t *)&ds->spec_n);
        hipLaunchKernelGGL(k_result, dim3(1), dim3(256), 0, c->stream, d_buf, c->rd.as<RecDesc>(),
                           c->mlist.as<uint32_t>(), 0u, ri, ds, c->h_res_dev, (const uint32_t *)&ds->spec_n,
                           (const uint8_t *)c->cat.as<uint8_t>());
        EW_CHECK(hipGetLastError());
        EW_CHECK(hipStreamSynchronize(c->stream));
        if (c->h_small->errflag) return EWAL_E_TIMEOUT;
        spec_checked = c->h_small->spec_n != 0;
        if (spec_checked) break;
      } else if ((rc = sync_small(c))) {
        return rc;
      }
      // k_frame declined before decoding anything: more candidates than
      // descriptors (a first call on record-dense WALs) or units with more
      // than EW_SLOTS candidates (small records) -> grow / k_rescan, run again
      const uint64_t Kf = c->h_small->total;
      const bool grow = Kf > rdcap && Kf <= ccap;
      const bool resc = c->h_small->novf && Kf <= ccap && !rescanned;
      if (ew_debug())
        std::fprintf(stderr, "ewal readall: general pass %d K %llu novf %u pos0 %llu irr %u spec %u\n", pass,
                     (unsigned long long)Kf, c->h_small->novf, (unsigned long long)c->h_small->pos0,
                     c->h_small->irregular, c->h_small->spec_n);
      if (!grow && !resc) break;
      if (resc) {
        if ((rc = ensure_cand_aux(c, ccap))) return rc;
        hipLaunchKernelGGL(k_rescan, dim3(64), dim3(256), 0, c->stream, d_buf, B, c->ovf.as<uint32_t>(), &ds->novf,
                           c->cbase.as<unsigned long long>(), c->cpos.as<uint64_t>(), c->clen.as<uint64_t>(), ccap);
        EW_CHECK(hipGetLastError());
        EW_CHECK(hipMemsetAsync(&ds->novf, 0, 4, c->stream));
        rescanned = true;
      }
      if (grow) rdcap = Kf + Kf / 8 + 1024;
    }
    K = c->h_small->total;
    if (ew_debug())
      std::fprintf(stderr, "ewal readall: fused_done %d K %llu novf %u pos0 %llu irr %u q %llu\n", (int)fused_done,
                   (unsigned long long)K, c->h_small->novf, (unsigned long long)c->h_small->pos0,
                   c->h_small->irregular, (unsigned long long)c->h_small->q);
    c->last_k = K;
    fused_done_final = fused_done;
    if (fused_done) {   // frames decoded and checked by k_frames; the result is in h_res
      decoded = true;
      spec_checked = true;
    } else if (K && K <= ccap && K <= rdcap && !c->h_small->novf && c->h_small->pos0 == 0 &&
               !c->h_small->irregular) {
      decoded = true;
      c->rd_valid = true;
      if (c->h_small->nslow && !spec_checked) {   // frames the canonical parser declined
        hipLaunchKernelGGL(k_decode_slow, dim3(std::min<uint64_t>(grid_for(c->h_small->nslow, 256), 1024)),
                           dim3(256), 0, c->stream, d_buf, B, c->cpos.as<uint64_t>(), (const uint32_t *)nullptr,
                           c->slow.as<uint32_t>(), ds, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice,
                           tb->shift, c->rd.as<RecDesc>(), pf, pf + rdcap, 0u, c->cat.as<uint8_t>(),
                           (uint64_t)c->cat.cap);
        EW_CHECK(hipGetLastError());
      }
    } else {
      // the speculation failed: frame by candidate links (k_link), growing
      // the candidate list first if it overflowed
      const unsigned lgrid = (unsigned)std::max(1, c->num_cu) * 8;
      if ((rc = ensure_cand_aux(c, ccap))) return rc;
      if (K <= ccap && c->h_small->novf) {   // candidates of the overflow units
        hipLaunchKernelGGL(k_rescan, dim3(64), dim3(256), 0, c->stream, d_buf, B, c->ovf.as<uint32_t>(), &ds->novf,
                           c->cbase.as<unsigned long long>(), c->cpos.as<uint64_t>(), c->clen.as<uint64_t>(), ccap);
        EW_CHECK(hipGetLastError());
      }
      if (K > ccap) {   // grow and redo the compaction (the slots stay valid)
        if (K >= 0xfffffff0ull) return EWAL_E_NOMEM;
        ccap = K + 1024;
        EW_CHECK(c->cpos.ensure(ccap * 8));
        rc = compact_cands(c, d_buf, B, (uint32_t)(B / EW_WAVE_BYTES + 1), ccap);
        if (rc) return rc;
      }
      EW_CHECK(hipMemsetAsync(&ds->irregular, 0, 4, c->stream));
      hipLaunchKernelGGL(k_link, dim3(lgrid), dim3(256), 0, c->stream, d_buf, B, c->cpos.as<uint64_t>(),
                         c->clen.as<uint64_t>(), ccap, c->nxt.as<uint32_t>(), c->exc.as<uint8_t>(), ds);
      EW_CHECK(hipGetLastError());
      if ((rc = sync_small(c))) return rc;
    }
  }
  out->n_candidates = (int64_t)K;
  JumpState js;
  uint32_t last_cand = EW_NIL;   // the chain's last candidate
  if (K && c->h_small->pos0 == 0) {
    if (!c->h_small->irregular) {
      regular = true;
      n = K;
      q = c->h_small->q;
      qlen = c->h_small->qlen;
      out->n_runs = 1;
      last_cand = (uint32_t)(K - 1);
    } else {
      rc = frame_irregular(c, K, out, &js, &n, &last_cand, &q);
      if (rc) return rc;
      rc = read_le64_at(c, d_buf, B, q, &qlen);
      if (rc) return rc;
    }
  } else {
    rc = read_le64_at(c, d_buf, B, 0, &qlen);   // frame 0 is not a candidate: the chain is empty
    if (rc) return rc;
  }
  int tst = classify_terminal(B, q, qlen);
  c->last_q = q;
  // The frame pass leaves no candidate list for k_walk: it declines such a
  // terminal itself (fc.rare 128).  Should that invariant ever break, the call
  // is redone on the general path, which walks the frame (round 4's r04b fault:
  // a batched shard ending in int64(3) + 3 bytes left k_decode a stale list).
  if (fused_done_final && tst == EWAL_FRAME_FITS) {
    const int f = c->fused;
    c->fused = 0;
    rc = readall_impl(c, d_buf, B, ri, out);
    c->fused = f;
    return rc;
  }
  // walked frames (not candidates) on the chain: decoded and checked with the
  // chain's candidates from one frame-position list (fpos)
  std::vector<uint64_t> xs;
  const uint64_t *fpos = nullptr;
  if (tst == EWAL_FRAME_FITS) {
    if (!K) {   // no candidate list at all: k_walk's search sees an empty one
      EW_CHECK(c->cpos.ensure(8));
    }
    rc = walk_chain(c, tb, d_buf, B, K, regular, &js, n ? last_cand : EW_NIL, &n, &q, &tst, xs);
    if (rc) return rc;
    const uint64_t nx = xs.size();
    if (nx) {
      const uint64_t nt = n + nx;
      if (nt >= 0xffffffffull) return EWAL_E_NOMEM;
      EW_CHECK(c->fpos.ensure((size_t)nt * 8));
      EW_CHECK(c->xpos.ensure((size_t)nx * 8));
      EW_CHECK(hipMemcpyAsync(c->xpos.p, xs.data(), (size_t)nx * 8, hipMemcpyHostToDevice, c->stream));
      const uint32_t *rcl = (regular || !js.ready) ? (const uint32_t *)nullptr : c->rec_cand.as<uint32_t>();
      hipLaunchKernelGGL(k_fpos, dim3(grid_for(nt, 256)), dim3(256), 0, c->stream, c->cpos.as<uint64_t>(), rcl,
                         (uint32_t)n, c->xpos.as<uint64_t>(), (uint32_t)nx, c->fpos.as<uint64_t>());
      // the frame list changed: decode and check it again from fresh reductions
      hipLaunchKernelGGL(k_reset_check, dim3(1), dim3(64), 0, c->stream, ds);
      EW_CHECK(hipGetLastError());
      fpos = c->fpos.as<uint64_t>();
      n = nt;
      decoded = false;
      spec_checked = false;
    }
  }

  c->last_q = q;   // (walk_chain may have moved it)
  ResultDev res;
  std::memset(&res, 0, sizeof(res));
  res.agg.first_fail = ~0ull;
  res.agg.last_entry = -1;
  res.agg.last_state = -1;
  res.agg.first_meta = ~0ull;
  if (n) {
    const uint32_t n32 = (uint32_t)n;
    if (!decoded) {
      if (n > c->pfcap) {
        EW_CHECK(c->rd.ensure((size_t)n * sizeof(RecDesc)));
        EW_CHECK(c->pf.ensure((size_t)n * 8));
        EW_CHECK(c->slow.ensure((size_t)n * 4));
        c->pfcap = n;
      }
      uint32_t *pf = c->pf.as<uint32_t>();
      const uint32_t *rc_list = (regular || fpos) ? (const uint32_t *)nullptr : c->rec_cand.as<uint32_t>();
      const uint64_t *plist = fpos ? fpos : c->cpos.as<uint64_t>();
      EW_CHECK(hipMemsetAsync(&ds->nslow, 0, 4, c->stream));
      c->rd_valid = true;
#ifdef EW_DEBUG_BOUNDS
      {   // tools/ debug builds: the frame list k_decode is about to read, checked on the host
        EW_CHECK(hipStreamSynchronize(c->stream));
        std::vector<uint32_t> rcl(rc_list ? n : 0);
        if (rc_list) EW_CHECK(hipMemcpy(rcl.data(), rc_list, n * 4, hipMemcpyDeviceToHost));
        const uint64_t pcap = (fpos ? c->fpos.cap : c->cpos.cap) / 8;
        std::vector<uint64_t> pl(pcap);
        EW_CHECK(hipMemcpy(pl.data(), plist, pcap * 8, hipMemcpyDeviceToHost));
        std::fprintf(stderr, "ewal dbg: n %llu K %llu regular %d fpos %d rc_list %d B %llu pcap %llu pfcap %llu "
                     "rdcap %zu q %llu\n", (unsigned long long)n, (unsigned long long)K, (int)regular, fpos != nullptr,
                     rc_list != nullptr, (unsigned long long)B, (unsigned long long)pcap,
                     (unsigned long long)c->pfcap, c->rd.cap / sizeof(RecDesc), (unsigned long long)q);
        {
          const uint64_t cc = std::min<uint64_t>(c->cpos.cap / 8, K + 4);
          std::vector<uint64_t> cp(cc);
          EW_CHECK(hipMemcpy(cp.data(), c->cpos.p, cc * 8, hipMemcpyDeviceToHost));
          std::fprintf(stderr, "ewal dbg: cpos");
          for (uint64_t i = 0; i < cc; ++i) std::fprintf(stderr, " %llu", (unsigned long long)cp[i]);
          std::fprintf(stderr, "\newal dbg: fpos");
          for (uint64_t i = 0; i < pcap; ++i) std::fprintf(stderr, " %llu", (unsigned long long)pl[i]);
          std::fprintf(stderr, "\newal dbg: xs");
          for (uint64_t x : xs) std::fprintf(stderr, " %llu", (unsigned long long)x);
          std::fprintf(stderr, "\n");
        }
        uint64_t prev = 0;
        for (uint64_t r = 0; r < n; ++r) {
          const uint64_t ix = rc_list ? rcl[r] : r;
          const uint64_t p = ix < pcap ? pl[ix] : ~0ull;
          if (ix >= pcap || p >= B || (r && p <= prev)) {
            std::fprintf(stderr, "ewal dbg: bad frame %llu: index %llu pos %llu prev %llu\n", (unsigned long long)r,
                         (unsigned long long)ix, (unsigned long long)p, (unsigned long long)prev);
            return EWAL_E_INVAL;
          }
          prev = p;
        }
      }
#endif
      // the list's capacities: k_decode checks every index it reads against them
      const uint64_t pcap = (fpos ? c->fpos.cap : c->cpos.cap) / 8;
      const uint64_t rccap = rc_list ? c->rec_cand.cap / 4 : 0;
      hipLaunchKernelGGL(k_decode, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, d_buf, B,
                         plist, pcap, rc_list, rccap, n32, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(),
                         tb->slice, tb->shift, c->rd.as<RecDesc>(), pf, pf + c->pfcap, c->slow.as<uint32_t>(), ds);
      hipLaunchKernelGGL(k_decode_slow, dim3(std::min<uint64_t>(grid_for(n, 256), 64)), dim3(256), 0, c->stream,
                         d_buf, B, plist, rc_list, c->slow.as<uint32_t>(), ds,
                         c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift, c->rd.as<RecDesc>(), pf,
                         pf + c->pfcap, n32, c->cat.as<uint8_t>(), (uint64_t)c->cat.cap);
    }
    RecDesc *rd = c->rd.as<RecDesc>();
    const uint32_t *pfd = c->pf.as<uint32_t>(), *pfo = pfd + c->pfcap;
    const uint32_t nb = grid_for(n, 1024);
    EW_CHECK(c->ops.ensure((size_t)n * 4));
    EW_CHECK(c->kk.ensure((size_t)n * 8));
    if (!spec_checked) {
      // look-back status words of k_check: zeroed when (re)allocated and when
      // the 24-bit epoch wraps; otherwise the epoch tells old words apart
      const size_t had = c->lbstat.cap;
      EW_CHECK(c->lbstat.ensure((size_t)nb * 8));
      c->epoch = (c->epoch + 1) & 0xffffffu;
      if (c->lbstat.cap != had || c->epoch == 0) {
        EW_CHECK(hipMemsetAsync(c->lbstat.p, 0, c->lbstat.cap, c->stream));
        if (c->epoch == 0) c->epoch = 1;
      }
      EW_CHECK(c->opf.ensure((size_t)nb * 4));   // k_check's per-workgroup op bases
      EW_CHECK(c->mlist.ensure((size_t)n * 4));
      EW_CHECK(c->ents.ensure((size_t)n * sizeof(ewal_entry)));
      EW_CHECK(c->ulist.ensure((size_t)n * sizeof(uint2)));
      SegArgs useg{};
      useg.ulist = c->ulist.as<uint2>();
      hipLaunchKernelGGL(k_check<false>, dim3(nb), dim3(1024), 0, c->stream, tb->shift, rd, n32, pfd, pfo, ri,
                         c->lbstat.as<unsigned long long>(), c->epoch, c->opf.as<uint32_t>(),
                         c->ents.as<ewal_entry>(), c->mlist.as<uint32_t>(), ds, useg, (const uint32_t *)nullptr);
      hipLaunchKernelGGL(k_result, dim3(1), dim3(256), 0, c->stream, d_buf, rd, c->mlist.as<uint32_t>(), n32, ri, ds,
                         c->h_res_dev, (const uint32_t *)nullptr, (const uint8_t *)c->cat.as<uint8_t>());
      EW_CHECK(hipGetLastError());
      EW_CHECK(hipStreamSynchronize(c->stream));
    }
    std::memcpy(&res, c->h_res, sizeof(ResultDev));
    if (res.errflag & EW_ERR_LIST) return EWAL_E_INVAL;
    if (res.errflag) return EWAL_E_TIMEOUT;
    if (res.gapslow || res.nonmono)   // the rare paths work on the op list
      hipLaunchKernelGGL(k_opslist, dim3(nb), dim3(1024), 0, c->stream, rd, n32, ri, c->opf.as<uint32_t>(),
                         c->ops.as<uint32_t>(), c->kk.as<uint64_t>());
    if (res.gapslow) {   // an op's predecessor lay too far back for k_check: list-based gap pass
      const unsigned ggrid = (unsigned)std::min<uint64_t>(grid_for(n, 256), (uint64_t)c->num_cu * 8);
      hipLaunchKernelGGL(k_gap, dim3(ggrid), dim3(256), 0, c->stream, rd, c->ops.as<uint32_t>(),
                         c->kk.as<uint64_t>(), ds);
      hipLaunchKernelGGL(k_result, dim3(1), dim3(256), 0, c->stream, d_buf, rd, c->mlist.as<uint32_t>(), n32, ri, ds,
                         c->h_res_dev, (const uint32_t *)nullptr, (const uint8_t *)c->cat.as<uint8_t>());
      EW_CHECK(hipGetLastError());
      EW_CHECK(hipStreamSynchronize(c->stream));
      std::memcpy(&res, c->h_res, sizeof(ResultDev));
    }
    out->n_slow = (int32_t)res.nslow;
    if (res.ncatfail && !c->cat_retry) {
      // a split byte field found no room in the side arena: grow it to what
      // the frames asked for and run the call again (once)
      EW_CHECK(c->cat.ensure((size_t)std::min<uint64_t>(2 * res.cat_need + (1 << 20), 2 * B + (1 << 20))));
      c->cat_retry = true;
      const int r2 = readall_impl(c, d_buf, B, ri, out);
      c->cat_retry = false;
      return r2;
    }
    c->cat_bytes = std::min<uint64_t>(res.cat_used, c->cat.cap);
  }
  const ReadAllAgg &hagg = res.agg;
  out->n_records = (int64_t)n;

  if (hagg.first_fail < n) {
    const RecDesc &f = res.fail;
    out->status = f.st;
    out->fail_record = (int64_t)hagg.first_fail;
    out->fail_offset = (int64_t)f.off;
    out->n_records = (int64_t)hagg.first_fail;
    if (f.st == EWAL_ERR_UNEXPECTED_TYPE) out->detail = f.type;
    if (f.st == EWAL_PANIC_INDEX_GAP) out->detail = (int64_t)f.f1;
  } else if (tst != EWAL_OK) {
    out->status = tst;
    out->fail_record = (int64_t)n;
    out->fail_offset = (int64_t)q;
  } else {
    const uint64_t enti = hagg.last_entry >= 0 ? res.lastent.f1 : 0;
    out->enti = enti;
    if (enti < ri) {
      out->status = EWAL_ERR_INDEX_NOT_FOUND;
      // (Go returns no lastCRC with this error; a range of a split WAL still
      // hands its running CRC to the next range, shard.split_verdict)
      if (n) out->last_crc = (c->defer_first && n == 1 && !fused_done_final && res.last.type != 4)
                                 ? res.last.crc : res.last.chained;
    } else {
      out->status = EWAL_OK;
      if (n) {
        out->last_crc = res.last.chained;
        // a deferred frame 0 that is the range's only frame: the running CRC
        // after it is its stored CRC once the caller's check holds (the
        // general path's descriptor keeps crc32.Update(0, Data) for the range
        // info; the fused pass reports the stored CRC itself)
        if (c->defer_first && n == 1 && !fused_done_final && res.last.type != 4) out->last_crc = res.last.crc;
        if (hagg.first_meta != ~0ull) {
          out->metadata_off = (int64_t)(res.md.pad0 == 2 ? rd_cat_off(res.md) : res.md.doff);
          out->metadata_len = (int64_t)res.md.dlen;
          if (res.md.pad0 == 2) out->flags |= EWAL_FLAG_METADATA_SPLIT;   // a range of the split bytes
        }
        if (hagg.last_state >= 0) {
          out->has_state = 1;
          out->state_term = res.sd.f0;
          out->state_vote = res.sd.f1;
          out->state_commit = res.sd.f2;
        }
        const uint32_t nops = res.nops;
        const uint64_t nents = nops ? res.klast + 1 : 0;
        out->n_ents = (int64_t)nents;
        if (nents && res.nonmono) {
          // index rewinds: op j is ents[k_j] iff every later op has k > k_j
          // (suffix-min over kk via a reversed inclusive min-scan)
          EW_CHECK(c->kkrev.ensure((size_t)nops * 8));
          EW_CHECK(c->suf.ensure((size_t)nops * 8));
          EW_CHECK(c->ents.ensure((size_t)nents * sizeof(ewal_entry)));
          uint64_t *kk = c->kk.as<uint64_t>();
          uint64_t *kr = c->kkrev.as<uint64_t>();
          uint64_t *sf = c->suf.as<uint64_t>();
          ev1_final = false;
          hipLaunchKernelGGL(k_reverse_u64, dim3(grid_for(nops, 256)), dim3(256), 0, c->stream, kk, kr, nops);
          size_t bytes = 0;
          EW_CHECK(hipcub::DeviceScan::InclusiveScan(nullptr, bytes, kr, sf, hipcub::Min(), (int)nops, c->stream));
          EW_CHECK(c->tmp.ensure(bytes));
          EW_CHECK(hipcub::DeviceScan::InclusiveScan(c->tmp.p, bytes, kr, sf, hipcub::Min(), (int)nops, c->stream));
          hipLaunchKernelGGL(k_reverse_u64, dim3(grid_for(nops, 256)), dim3(256), 0, c->stream, sf, kr, nops);
          hipLaunchKernelGGL(k_ents, dim3(grid_for(nops, 256)), dim3(256), 0, c->stream, c->rd.as<RecDesc>(),
                             c->ops.as<uint32_t>(), nops, kk, kr, c->ents.as<ewal_entry>(), nents);
          EW_CHECK(hipGetLastError());
        }
        c->last_nents = nents;
        if (res.nunrec || (hagg.last_state >= 0 && res.sd.pad1)) {
          ev1_final = false;
          rc = gather_unrec(c, d_buf, res, hagg, nents);
          if (rc) return rc;
          out->n_unrec = (uint32_t)c->unrec.size();
        }
      }
      c->last_ok = true;
    }
  }
  if (fused_done_final) out->flags |= EWAL_FLAG_FAST_PATH;
  c->last_n = n;
  if (B) c->dense_hint = n * EW_WAVE_BYTES >= 4 * B;   // >= 4 frames per 4 KiB unit: the next call stores vh[]
  c->rec_rebuild = n && !c->rd_valid;   // the fused pass decided: descriptors are rebuilt on demand
  c->rec_valid = true;
  if (!ev1_final) EW_CHECK(hipEventRecord(c->ev1, c->stream));
  EW_CHECK(hipEventSynchronize(c->ev1));
  if (B) {
    if (int rc2 = set_times(c, out)) return rc2;
  } else {
    float ms = 0;
    EW_CHECK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    out->device_ms = ms;
  }
  return out->status;
}

// Grow-only device buffer that keeps its first `keep` bytes.
static hipError_t grow_keep(DevBuf &b, size_t need, size_t keep, hipStream_t st) {
  if (need <= b.cap) return hipSuccess;
  DevBuf nb;
  hipError_t e = nb.ensure(std::max(need, b.cap * 2));
  if (e != hipSuccess) return e;
  if (keep) {
    e = hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      nb.release();
      return e;
    }
  }
  b.adopt(nb);
  return hipSuccess;
}

// The batch on the frame pass (k_shard_nfp / k_shard_rbase: every shard's
// ents region; k_frames<true>, k_frames_seam<true>; per-shard metadata rule
// and results): ONE host sync.  *done when the pass decided the batch (out[]
// and the ents / ent_first tables filled; shards it could not decide carry
// EW_SHARD_BAD); otherwise the caller runs the general batch path.  Shard s's
// entry op k is bents[rbase[s] + k], rbase[s] = 4 x the flagged pieces of the
// shards before s (an entry frame is >= 20 bytes: at most 4 start in a 64-B
// piece); *have = the regions' total (shards replayed alone append after it).
// frames per 4 KiB unit from which a batch's next stream pass stores vh[]
// (the 128-B prefixes of the batch frame pass; round 6, profiles/r06/)
#ifndef EW_VH_BATCH_FPU
#define EW_VH_BATCH_FPU 3
#endif
static int frames_batch(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, uint32_t ns,
                        const std::vector<uint64_t> &soff, const uint64_t *ris, ewal_result *out, bool *done,
                        uint64_t *have) {
  Small *ds = c->small.as<Small>();
  *done = false;
  const uint32_t nunits = (uint32_t)(B / EW_WAVE_BYTES + 1);
  const int tsh = fr_tsh(c, nunits);
  const uint32_t tu = 1u << tsh, ntiles = (nunits + tu - 1) / tu;
  if (int rc = fr_ensure(c, nunits, ntiles)) return rc;
  EW_CHECK(c->bsoff.ensure((size_t)(ns + 1) * 8));
  EW_CHECK(c->bri.ensure((size_t)ns * 8));
  EW_CHECK(c->bres.ensure((size_t)ns * sizeof(ewal_result)));
  EW_CHECK(c->bef.ensure((size_t)ns * 8));
  EW_CHECK(c->fnfp.ensure((size_t)ns * 8));
  EW_CHECK(c->frbase.ensure((size_t)(ns + 1) * 8));
  EW_CHECK(c->fsp.ensure((size_t)ns * sizeof(ShardPos)));
  EW_CHECK(c->ftcb.ensure((size_t)ntiles * 4));
  EW_CHECK(hipMemcpyAsync(c->bsoff.p, soff.data(), (size_t)(ns + 1) * 8, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipMemcpyAsync(c->bri.p, ris, (size_t)ns * 8, hipMemcpyHostToDevice, c->stream));
  FrSeg sg;
  sg.ns = ns;
  sg.soff = c->bsoff.as<uint64_t>();
  sg.ri = c->bri.as<uint64_t>();
  sg.rbase = c->frbase.as<uint64_t>();
  sg.sp = c->fsp.as<ShardPos>();
  sg.tcb = c->ftcb.as<uint32_t>();
  uint64_t ecap = std::max<uint64_t>(c->bents.cap / sizeof(ewal_entry), B / 256 + 1024);
  uint32_t mcap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(c->mlist.cap / 8, (uint64_t)ns + 4096), 0xffffffffull);
  // the shards the ctx's previous batch of this shape saw rewind: rewind mode in this pass
  const bool hint = !c->brew_hint.empty() && c->brew_ns == ns && c->brew_B == B;
  const uint32_t nhint = hint ? (uint32_t)c->brew_hint.size() : 0u;
  if (hint) {
    EW_CHECK(c->fhint.ensure((size_t)nhint * 4));
    EW_CHECK(hipMemcpyAsync(c->fhint.p, c->brew_hint.data(), (size_t)nhint * 4, hipMemcpyHostToDevice, c->stream));
  }
  for (int pass = 0; pass < 3; ++pass) {
    EW_CHECK(grow_keep(c->bents, (size_t)ecap * sizeof(ewal_entry), 0, c->stream));
    EW_CHECK(c->mlist.ensure((size_t)mcap * 8));
    if (pass) if (int rc = reset_small(c)) return rc;
    FrArgs a = fr_args(c, tb, d_buf, B, nunits, ntiles, 0, c->bents.as<ewal_entry>(), ecap, mcap);
    a.vh = c->ov_sa.vh;   // the batch's stream pass stored vh[] (record-dense shards): the 128-B prefixes
    if (hint) {
      EW_CHECK(c->fown.ensure((size_t)ecap * 8));
      EW_CHECK(c->fcl.ensure((size_t)c->brew_clcap * 4));
      a.rew = 1;
      a.own = c->fown.as<unsigned long long>();
      a.clist = c->fcl.as<uint32_t>();
      a.ccap = c->brew_clcap;
    }
    const unsigned ngrid = (unsigned)std::min<uint64_t>(ns, (uint64_t)std::max(1, c->num_cu) * 4);
    hipLaunchKernelGGL(k_shard_nfp, dim3(ngrid), dim3(256), 0, c->stream, a.hmask, nunits, sg.soff, ns,
                       c->fnfp.as<unsigned long long>());
    hipLaunchKernelGGL(k_shard_rbase, dim3(1), dim3(1024), 0, c->stream, (const unsigned long long *)c->fnfp.p, ns,
                       ecap, sg.rbase, sg.sp, ds);
    if (hint)
      hipLaunchKernelGGL(k_shard_hint, dim3(std::min<uint32_t>(nhint, 256)), dim3(256), 0, c->stream, sg.sp,
                         (const uint32_t *)c->fhint.as<uint32_t>(), nhint, (const uint64_t *)sg.rbase, a.own,
                         (const Small *)ds);
    EW_CHECK(hipEventRecord(c->evf0, c->stream));
    c->evf_start = c->evf0;
    fr_launch_frames<true>(tsh, ntiles, a, sg, fr_cus(c), c->stream);
    EW_CHECK(hipEventRecord(c->evf1, c->stream));
    fr_launch_seam<true>(c, tsh, ntiles, a, sg, nullptr, nullptr);
    if (hint)   // the hinted shards' slots claimed twice: their last op's entry
      hipLaunchKernelGGL(k_ents_fix, dim3((unsigned)std::max(1, c->num_cu) * 2), dim3(256), 0, c->stream, d_buf, B,
                         (const unsigned long long *)a.own, (const uint32_t *)a.clist, a.ccap, (const Small *)ds,
                         a.ents, (const uint64_t *)sg.soff, ns);
    c->frames_timed = true;
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, c->stream, (const uint32_t *)a.tcnt, ntiles, sg.tcb,
                       (const Small *)ds);
    hipLaunchKernelGGL(k_meta_batch_fr, dim3(64), dim3(256), 0, c->stream, a, sg);
    fr_launch_result_batch(c, tsh, a, sg);
    hipLaunchKernelGGL(k_batch_gate_fr, dim3(1), dim3(64), 0, c->stream, ds, c->h_small_dev);
    EW_CHECK(hipGetLastError());
    EW_CHECK(hipMemcpyAsync(out, c->bres.p, (size_t)ns * sizeof(ewal_result), hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipMemcpyAsync(c->bent_first.data(), c->bef.p, (size_t)ns * 8, hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipEventRecord(c->ev1, c->stream));
    EW_CHECK(ew_sync(c));
    const Small *hs = c->h_small;
    if (hs->errflag) return EWAL_E_TIMEOUT;
    c->last_k = hs->total;
    c->dense_hint_batch = hs->total * EW_WAVE_BYTES >= (uint64_t)EW_VH_BATCH_FPU * B;
    if (hs->spec_n) {
      if (int rc = set_times(c, out, ns)) return rc;
      for (uint32_t i = 0; i < ns; ++i) {
        c->bnents[i] = (uint64_t)out[i].n_ents;
        if (!out[i].n_ents) c->bent_first[i] = 0;
      }
      *have = hs->fr_need;
      *done = true;
      return 0;
    }
    bool again = false;
    if (hs->fr_capfail && hs->fr_need > ecap) {
      ecap = hs->fr_need + hs->fr_need / 8 + 1024;
      again = true;
    }
    if ((hs->fc.rare & 8u) && hs->nmeta > mcap) {
      mcap = hs->nmeta + hs->nmeta / 8 + 1024;
      again = true;
    }
    if ((hs->fc.rare & 64u) && hint) {   // more slots claimed twice than the list holds: once more
      c->brew_clcap = (uint32_t)std::min<uint64_t>((uint64_t)hs->fr_ncl + hs->fr_ncl / 8 + 1024, 0xffffffffull);
      again = true;
    }
    if (!again || (hs->fc.rare & ~(8u | 64u))) break;
  }
  return 0;
}

// The batch's shards whose entry indexes go back (leader changes: ReadAll's
// ents = append(ents[:Index-ri], e) truncates, wal/wal.go:173): their
// verdicts from the batch's pass stand (k_result_batch_fr), only the ents
// slots more than one op wrote are fixed -- k_rew_claim claims every op's
// slot over the shards' 64 KiB tiles, k_ents_fix stores the last op's entry
// in the slots claimed twice.  (Round 4 reran the whole frame pass over the
// shards' 1 MiB tiles, one wave each: 1.07x the clean batch for 5 shards.)
static int frames_batch_rewind(ewal_ctx *c, DevTables *tb, const uint8_t *d_buf, uint64_t B, uint32_t ns,
                               const std::vector<uint64_t> &soff, const std::vector<uint32_t> &rews, ewal_result *out,
                               uint64_t have) {
  (void)tb;
  Small *ds = c->small.as<Small>();
  const uint32_t nunits = (uint32_t)(B / EW_WAVE_BYTES + 1);
  const uint64_t tb_bytes = (uint64_t)REW_TU * EW_WAVE_BYTES;
  const uint32_t ntiles = (nunits + REW_TU - 1) / REW_TU;
  std::vector<uint64_t> rbase(ns + 1);
  EW_CHECK(hipMemcpy(rbase.data(), c->frbase.p, (size_t)(ns + 1) * 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> tiles;
  std::vector<uint8_t> smask(ns, 0);
  uint64_t slots = 0;
  for (uint32_t s : rews) {
    if (soff[s + 1] == soff[s]) continue;
    smask[s] = 1;
    slots += rbase[s + 1] - rbase[s];
    for (uint64_t t = soff[s] / tb_bytes; t <= (soff[s + 1] - 1) / tb_bytes && t < ntiles; ++t)
      if (tiles.empty() || tiles.back() < t) tiles.push_back((uint32_t)t);
  }
  if (tiles.empty()) return 0;
  std::sort(tiles.begin(), tiles.end());
  tiles.erase(std::unique(tiles.begin(), tiles.end()), tiles.end());
  const uint32_t ntl = (uint32_t)tiles.size();
  uint32_t clcap = (uint32_t)std::min<uint64_t>(slots + 1024, 0xffffffffull);
  EW_CHECK(c->fown.ensure((size_t)std::max<uint64_t>(have, 1) * 8));
  EW_CHECK(c->ftl.ensure((size_t)ntl * 4 + ns + 16));
  uint32_t *d_tl = c->ftl.as<uint32_t>();
  uint8_t *d_sm = (uint8_t *)(d_tl + ntl);
  EW_CHECK(hipMemcpyAsync(d_tl, tiles.data(), (size_t)ntl * 4, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipMemcpyAsync(d_sm, smask.data(), ns, hipMemcpyHostToDevice, c->stream));
  const unsigned grid = (unsigned)std::min<uint64_t>(grid_for(ntl, 4), (uint64_t)std::max(1, c->num_cu) * 8);
  for (int pass = 0; pass < 2; ++pass) {
    EW_CHECK(c->fcl.ensure((size_t)clcap * 4));
    for (uint32_t s : rews)   // the shards' regions unclaimed
      if (smask[s])
        EW_CHECK(hipMemsetAsync(c->fown.as<unsigned long long>() + rbase[s], 0,
                                (size_t)(rbase[s + 1] - rbase[s]) * 8, c->stream));
    EW_CHECK(hipMemsetAsync(&ds->fr_ncl, 0, 4, c->stream));
    hipLaunchKernelGGL(k_rew_claim, dim3(grid), dim3(256), 0, c->stream, d_buf, B, nunits,
                       (const ulonglong2 *)c->hmask.as<unsigned long long>(), (const uint32_t *)d_tl, ntl,
                       c->bsoff.as<uint64_t>(), ns, c->bri.as<uint64_t>(), c->frbase.as<uint64_t>(),
                       (const uint8_t *)d_sm, c->fown.as<unsigned long long>(), c->fcl.as<uint32_t>(), clcap, ds);
    hipLaunchKernelGGL(k_ents_fix, dim3((unsigned)std::max(1, c->num_cu) * 2), dim3(256), 0, c->stream, d_buf, B,
                       (const unsigned long long *)c->fown.as<unsigned long long>(), (const uint32_t *)c->fcl.as<uint32_t>(),
                       clcap, (const Small *)ds, c->bents.as<ewal_entry>(), (const uint64_t *)c->bsoff.as<uint64_t>(), ns);
    EW_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_export_small, dim3(1), dim3(64), 0, c->stream, ds, c->h_small_dev);
    EW_CHECK(hipEventRecord(c->ev1, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
    const Small *hs = c->h_small;
    if (hs->errflag) return EWAL_E_TIMEOUT;
    if (!(hs->fc.rare & 64u)) break;
    clcap = hs->fr_ncl + hs->fr_ncl / 8 + 1024;   // more slots claimed twice than listed: once more
    EW_CHECK(hipMemsetAsync(&ds->fc.rare, 0, 4, c->stream));
  }
  if (c->h_small->fc.rare) {   // (not decided: every listed shard replayed alone)
    for (uint32_t s : rews) out[s].flags = EW_SHARD_BAD;
    return 0;
  }
  return set_times(c, out, ns);
}

// ReadAll of the listed shards of a batch, each alone (readall_impl over an
// aligned scratch copy: the stream pass reads 16-B aligned): shards the
// fused pass could not decide (torn or corrupt framing, index rewinds,
// encodings the canonical parser declines, unknown fields) or the whole
// batch when the general path could not decide it.  Their ents are appended
// to bents after the first `have` entries; their XXX_unrecognized side lists
// are kept per shard (ewal_batch_copy_unrec).  device_ms of every result
// becomes the batch's plus the replays'.
static int replay_shards(ewal_ctx *c, const uint8_t *d_buf, const std::vector<uint64_t> &soff, const uint64_t *lens,
                         const uint64_t *ris, ewal_result *out, const std::vector<uint32_t> &which, uint64_t have) {
  const uint32_t ns = (uint32_t)soff.size() - 1;
  c->bunrec.assign(ns, {});
  c->bunrec_bytes.assign(ns, {});
  c->bsplit_bytes.assign(ns, {});
  if (which.empty()) return 0;
  const uint64_t keep_k = c->last_k;
  const double batch_ms = ns ? out[0].device_ms : 0.0, batch_stream = ns ? out[0].stream_ms : 0.0;
  double extra = 0;
  for (uint32_t i : which) {
    const uint8_t *p = d_buf;
    if (lens[i]) {
      EW_CHECK(c->bshard.ensure(lens[i] + 64));
      EW_CHECK(hipMemcpyAsync(c->bshard.p, d_buf + soff[i], lens[i], hipMemcpyDeviceToDevice, c->stream));
      p = c->bshard.as<uint8_t>();
    }
    ewal_result r;
    int rc = readall_impl(c, p, lens[i], ris[i], &r);
    if (rc < 0) return rc;
    extra += r.device_ms;
    r.flags |= EWAL_FLAG_SHARD_FALLBACK;
    if (r.status == EWAL_OK && r.n_unrec) {
      c->bunrec[i] = c->unrec;
      c->bunrec_bytes[i].resize(c->unrec_bytes);
      if (c->unrec_bytes)
        EW_CHECK(hipMemcpy(c->bunrec_bytes[i].data(), c->uarena.p, c->unrec_bytes, hipMemcpyDeviceToHost));
    }
    if (r.status == EWAL_OK && c->cat_bytes) {   // split byte fields: the ents / metadata views index these
      c->bsplit_bytes[i].resize(c->cat_bytes);
      EW_CHECK(hipMemcpy(c->bsplit_bytes[i].data(), c->cat.p, c->cat_bytes, hipMemcpyDeviceToHost));
    }
    const uint64_t ne = r.status == EWAL_OK ? (uint64_t)r.n_ents : 0;
    c->bent_first[i] = 0;
    c->bnents[i] = 0;
    if (ne) {
      EW_CHECK(grow_keep(c->bents, (size_t)(have + ne) * sizeof(ewal_entry), (size_t)have * sizeof(ewal_entry),
                         c->stream));
      EW_CHECK(hipMemcpyAsync(c->bents.as<ewal_entry>() + have, c->ents.p, (size_t)ne * sizeof(ewal_entry),
                              hipMemcpyDeviceToDevice, c->stream));
      c->bent_first[i] = have;
      c->bnents[i] = ne;
      have += ne;
    }
    out[i] = r;
  }
  EW_CHECK(hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < ns; ++i) {
    out[i].device_ms = batch_ms + extra;
    if (out[i].flags & EWAL_FLAG_SHARD_FALLBACK) out[i].stream_ms = batch_stream;
  }
  c->last_k = keep_k;
  return 0;
}

// Batched ReadAll over many independent WALs (per-raft-group shards, SURVEY
// §8(d) C3) laid end to end in one device buffer: ONE stream pass, ONE frame
// pass and ONE segmented check (k_check<true>) for the whole batch, two host
// syncs in all, instead of a pipeline per shard.  The batch's frame chain runs
// through every shard when each ends on a frame boundary; when it does not
// (a torn or corrupt frame boundary), or on the rare op-list paths (index
// rewinds, far-back gap predecessors), the shards are verified one by one
// through readall_impl (result flag EWAL_FLAG_SHARD_FALLBACK).
static int readall_batch_impl(ewal_ctx *c, const uint8_t *d_buf, uint32_t ns, const uint64_t *lens,
                              const uint64_t *ris, ewal_result *out) {
  std::vector<uint64_t> soff(ns + 1, 0);
  for (uint32_t i = 0; i < ns; ++i) {
    soff[i + 1] = soff[i] + lens[i];
    if (soff[i + 1] < soff[i]) return EWAL_E_INVAL;
  }
  const uint64_t B = soff[ns];
  if (((uintptr_t)d_buf & 15) != 0 && B) return EWAL_E_INVAL;
  c->bent_first.assign(ns, 0);
  c->bnents.assign(ns, 0);
  c->last_ok = false;
  c->last_n = 0;
  c->last_nents = 0;
  DevTables *tb;
  int rc = get_tables(c, 0x82F63B78u, &tb);
  if (rc) return rc;
  EW_CHECK(c->small.ensure(sizeof(Small)));
  Small *ds = c->small.as<Small>();
  bool fast = B > 0 && ns > 0;
  float dev_ms = 0, str_ms = 0;
  if (fast) {
    EW_CHECK(hipEventRecord(c->ev0, c->stream));
    const uint64_t ccap = cand_cap(B);
    EW_CHECK(c->cpos.ensure(ccap * 8));
    uint64_t rdcap = std::min<uint64_t>(ccap, std::max<uint64_t>(c->last_k + c->last_k / 8 + 1024,
                                                                 B / 1024 + 1024));
    // record-dense shards (the ctx's previous batch: >= EW_VH_BATCH_FPU frames
    // per 4 KiB unit, or EWAL_OPT_VH_ON): the stream pass also stores vh[] and
    // the batch's frame pass takes its prefixes from 128-B boundaries
    const bool vh = c->fused && (c->vh_opt > 0 || (c->vh_opt == 0 && c->dense_hint_batch));
    if (vh) {
      EW_CHECK(c->vhb.ensure(((size_t)B / EW_WAVE_BYTES + 1) * EW_VPU * 4));
      c->vh_next = c->vhb.as<uint32_t>();
    }
    rc = run_stream(c, tb, d_buf, B, 1, ccap, !c->fused);
    if (rc) return rc;
#if EW_XS
    // timing-only ablation builds (tools/build_ab.sh -DEW_XS=...): the stream pass alone
    EW_CHECK(hipEventRecord(c->ev1, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
    EW_CHECK(hipEventElapsedTime(&dev_ms, c->ev0, c->ev1));
    EW_CHECK(hipEventElapsedTime(&str_ms, c->evs0, c->evs1));
    for (uint32_t i = 0; i < ns; ++i) {
      std::memset(&out[i], 0, sizeof(out[i]));
      out[i].device_ms = dev_ms;
      out[i].stream_ms = str_ms;
    }
    return 0;
#endif
    if (c->fused) {
      bool done = false;
      uint64_t have = 0;
      rc = frames_batch(c, tb, d_buf, B, ns, soff, ris, out, &done, &have);
      if (rc) return rc;
      if (ew_debug()) {
        uint32_t nb = 0;
        for (uint32_t i = 0; i < ns && done; ++i) nb += (out[i].flags & EW_SHARD_BAD) != 0;
        std::fprintf(stderr, "ewal batch: frame pass done %d bad %u (K %llu need %llu rare %u irr %u capfail %u err %u)\n",
                     (int)done, nb, (unsigned long long)c->h_small->total, (unsigned long long)c->h_small->fr_need,
                     c->h_small->fc.rare, c->h_small->irregular, c->h_small->fr_capfail, c->h_small->errflag);
      }
      if (done) {   // every shard decided but those the fused pass flagged: they are replayed alone
        std::vector<uint32_t> rews;
        c->brew_hint.clear();   // the next batch of this shape: these shards in rewind mode
        for (uint32_t i = 0; i < ns; ++i) {
          if (out[i].flags & EW_SHARD_BAD) continue;
          if (out[i].flags & EW_SHARD_REW) rews.push_back(i);
          if (out[i].flags & (EW_SHARD_REW | EW_SHARD_REWIN)) c->brew_hint.push_back(i);
        }
        c->brew_ns = ns;
        c->brew_B = B;
        if (!rews.empty() && (rc = frames_batch_rewind(c, tb, d_buf, B, ns, soff, rews, out, have))) return rc;
        for (uint32_t i = 0; i < ns; ++i) out[i].flags &= ~(EW_SHARD_REW | EW_SHARD_REWIN);
        std::vector<uint32_t> bad;
        for (uint32_t i = 0; i < ns; ++i)
          if (out[i].flags & EW_SHARD_BAD) bad.push_back(i);
        if (bad.empty()) {
          c->bunrec.assign(ns, {});
          c->bunrec_bytes.assign(ns, {});
          c->bsplit_bytes.assign(ns, {});
          return 0;
        }
        rc = replay_shards(c, d_buf, soff, lens, ris, out, bad, have);
        if (rc) return rc;
        forget_records(c);
        return 0;
      }
      // the general batch path over the same stream pass: its candidates and prefixes first
      if ((rc = reset_small(c))) return rc;
      if ((rc = run_cand_scan(c, tb, d_buf, B, 1, ccap))) return rc;
    }
    uint32_t *pf = nullptr;
    bool rescanned = false;
    for (int pass = 0; pass < 3; ++pass) {
      EW_CHECK(c->rd.ensure(rdcap * sizeof(RecDesc)));
      EW_CHECK(c->pf.ensure(rdcap * 8));
      EW_CHECK(c->slow.ensure(rdcap * 4));
      c->pfcap = rdcap;
      pf = c->pf.as<uint32_t>();
      const unsigned fgrid = (unsigned)std::max(1, c->num_cu) * c->frame_wg;
      hipLaunchKernelGGL(k_frame, dim3(fgrid), dim3(256), 0, c->stream, d_buf, B, c->cpos.as<uint64_t>(), ccap,
                         rdcap, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift,
                         c->rd.as<RecDesc>(), pf, pf + rdcap, c->slow.as<uint32_t>(), ds, c->ablate);
      EW_CHECK(hipGetLastError());
      if ((rc = sync_small(c))) return rc;
      // k_frame declined before decoding anything when there were more
      // candidates than descriptors or units with more than EW_SLOTS
      // candidates (small records): grow / k_rescan, and run it again
      const uint64_t Kf = c->h_small->total;
      const bool grow = Kf > rdcap && Kf <= ccap;
      const bool resc = c->h_small->novf && Kf <= ccap && !rescanned;
      if (!grow && !resc) break;
      if (resc) {
        if ((rc = ensure_cand_aux(c, ccap))) return rc;
        hipLaunchKernelGGL(k_rescan, dim3(64), dim3(256), 0, c->stream, d_buf, B, c->ovf.as<uint32_t>(), &ds->novf,
                           c->cbase.as<unsigned long long>(), c->cpos.as<uint64_t>(), c->clen.as<uint64_t>(), ccap);
        EW_CHECK(hipGetLastError());
        EW_CHECK(hipMemsetAsync(&ds->novf, 0, 4, c->stream));
        rescanned = true;
      }
      if (grow) rdcap = Kf + Kf / 8 + 1024;
    }
    const uint64_t K = c->h_small->total;
    c->last_k = K;
    fast = K && K <= ccap && K <= rdcap && !c->h_small->novf && c->h_small->pos0 == 0 && !c->h_small->irregular &&
           c->h_small->q == B;
    if (!fast && ew_debug())
      std::fprintf(stderr, "ewal batch: one by one (K %llu ccap %llu rdcap %llu novf %u pos0 %llu irr %u q %llu B %llu)\n",
                   (unsigned long long)K, (unsigned long long)ccap, (unsigned long long)rdcap, c->h_small->novf,
                   (unsigned long long)c->h_small->pos0, c->h_small->irregular, (unsigned long long)c->h_small->q,
                   (unsigned long long)B);
    if (fast) {
      const uint32_t n32 = (uint32_t)K;
      if (c->h_small->nslow) {
        hipLaunchKernelGGL(k_decode_slow, dim3(std::min<uint64_t>(grid_for(c->h_small->nslow, 256), 1024)),
                           dim3(256), 0, c->stream, d_buf, B, c->cpos.as<uint64_t>(), (const uint32_t *)nullptr,
                           c->slow.as<uint32_t>(), ds, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice,
                           tb->shift, c->rd.as<RecDesc>(), pf, pf + rdcap, 0u, (uint8_t *)nullptr, 0ull);
        EW_CHECK(hipGetLastError());
      }
      EW_CHECK(c->bsoff.ensure((size_t)(ns + 1) * 8));
      EW_CHECK(c->bri.ensure((size_t)ns * 8));
      EW_CHECK(c->bfs.ensure((size_t)(ns + 1) * 4));
      EW_CHECK(c->bsagg.ensure((size_t)ns * sizeof(ShardAgg)));
      EW_CHECK(c->bres.ensure((size_t)ns * sizeof(ewal_result)));
      EW_CHECK(c->bef.ensure((size_t)ns * 8));
      EW_CHECK(hipMemcpyAsync(c->bsoff.p, soff.data(), (size_t)(ns + 1) * 8, hipMemcpyHostToDevice, c->stream));
      EW_CHECK(hipMemcpyAsync(c->bri.p, ris, (size_t)ns * 8, hipMemcpyHostToDevice, c->stream));
      RecDesc *rd = c->rd.as<RecDesc>();
      hipLaunchKernelGGL(k_shard_start, dim3(grid_for(ns + 1, 256)), dim3(256), 0, c->stream, rd, n32,
                         c->bsoff.as<uint64_t>(), ns, c->bfs.as<uint32_t>(), c->bsagg.as<ShardAgg>(), ds);
      const uint32_t nb = grid_for(K, 1024);
      const size_t had = c->lbstat.cap;
      EW_CHECK(c->lbstat.ensure((size_t)nb * 8));
      c->epoch = (c->epoch + 1) & 0xffffffu;
      if (c->lbstat.cap != had || c->epoch == 0) {
        EW_CHECK(hipMemsetAsync(c->lbstat.p, 0, c->lbstat.cap, c->stream));
        if (c->epoch == 0) c->epoch = 1;
      }
      EW_CHECK(c->opf.ensure((size_t)nb * 4));
      EW_CHECK(c->mlist.ensure((size_t)K * 4));
      EW_CHECK(grow_keep(c->bents, (size_t)K * sizeof(ewal_entry), 0, c->stream));
      EW_CHECK(c->ulist.ensure((size_t)K * sizeof(uint2)));
      SegArgs sg;
      sg.ulist = c->ulist.as<uint2>();
      sg.fs = c->bfs.as<uint32_t>();
      sg.ns = ns;
      sg.ri = c->bri.as<uint64_t>();
      sg.soff = c->bsoff.as<uint64_t>();
      sg.sagg = c->bsagg.as<ShardAgg>();
      hipLaunchKernelGGL(k_check<true>, dim3(nb), dim3(1024), 0, c->stream, tb->shift, rd, n32, pf, pf + rdcap, 0ull,
                         c->lbstat.as<unsigned long long>(), c->epoch, c->opf.as<uint32_t>(),
                         c->bents.as<ewal_entry>(), c->mlist.as<uint32_t>(), ds, sg, (const uint32_t *)nullptr);
      hipLaunchKernelGGL(k_meta_batch, dim3(64), dim3(256), 0, c->stream, d_buf, rd, c->mlist.as<uint32_t>(), ds, sg);
      hipLaunchKernelGGL(k_result_batch, dim3(grid_for(ns, 256)), dim3(256), 0, c->stream, rd, sg,
                         c->bres.as<ewal_result>(), c->bef.as<unsigned long long>());
      EW_CHECK(hipGetLastError());
      EW_CHECK(hipMemcpyAsync(out, c->bres.p, (size_t)ns * sizeof(ewal_result), hipMemcpyDeviceToHost, c->stream));
      EW_CHECK(hipMemcpyAsync(c->bent_first.data(), c->bef.p, (size_t)ns * 8, hipMemcpyDeviceToHost, c->stream));
      EW_CHECK(hipEventRecord(c->ev1, c->stream));
      if ((rc = sync_small(c))) return rc;
      // split byte fields (no side arena in the batch) go one by one too
      fast = !c->h_small->segbad && !c->h_small->gapslow && !c->h_small->nonmono && !c->h_small->nunrec &&
             !c->h_small->ncatfail;
      if (!fast && ew_debug())
        std::fprintf(stderr, "ewal batch: one by one (segbad %u gapslow %u nonmono %u nunrec %u)\n",
                     c->h_small->segbad, c->h_small->gapslow, c->h_small->nonmono, c->h_small->nunrec);
      if (fast) {
        EW_CHECK(hipEventElapsedTime(&dev_ms, c->ev0, c->ev1));
        EW_CHECK(hipEventElapsedTime(&str_ms, c->evs0, c->evs1));
        c->bunrec.assign(ns, {});
        c->bunrec_bytes.assign(ns, {});
        c->bsplit_bytes.assign(ns, {});
        for (uint32_t i = 0; i < ns; ++i) {
          out[i].device_ms = dev_ms;
          out[i].stream_ms = str_ms;
          out[i].n_slow = (int32_t)c->h_small->nslow;
          c->bnents[i] = (uint64_t)out[i].n_ents;
          if (!out[i].n_ents) c->bent_first[i] = 0;
        }
        return 0;
      }
    }
  }
  // one shard at a time (the general path could not decide the batch)
  c->bent_first.assign(ns, 0);
  c->bnents.assign(ns, 0);
  std::vector<uint32_t> all(ns);
  for (uint32_t i = 0; i < ns; ++i) all[i] = i;
  rc = replay_shards(c, d_buf, soff, lens, ris, out, all, 0);
  if (rc) return rc;
  c->last_ok = false;
  forget_records(c);   // the descriptors of the last one-by-one shard are not a ReadAll of the batch
  return 0;
}

// The per-frame descriptors of the last ReadAll when the fused pass decided
// it (it keeps none in HBM): the general path's frame pass and check over the
// same stream pass (still in the ctx), for ewal_copy_records.
static int materialise_records(ewal_ctx *c) {
  const uint64_t n = c->last_n;
  DevTables *tb;
  int rc = get_tables(c, 0x82F63B78u, &tb);
  if (rc) return rc;
  Small *ds = c->small.as<Small>();
  const uint64_t ccap = std::min<uint64_t>(c->last_B / 128 + 65536, 0xfffffff0ull);
  EW_CHECK(c->rd.ensure((size_t)n * sizeof(RecDesc)));
  EW_CHECK(c->pf.ensure((size_t)n * 8));
  EW_CHECK(c->slow.ensure((size_t)n * 4));
  c->pfcap = n;
  uint32_t *pf = c->pf.as<uint32_t>();
  if (!c->scan_valid) {   // the frame pass decided the call: the candidate list and prefixes first
    EW_CHECK(hipMemsetAsync(ds, 0, sizeof(Small), c->stream));
    if (c->last_deferred) EW_CHECK(hipMemsetAsync(&ds->defer_first, 1, 1, c->stream));
    if ((rc = run_cand_scan(c, tb, c->last_buf, c->last_B, 1, ccap))) return rc;
    if ((rc = sync_small(c))) return rc;
    if (c->h_small->novf && (rc = rescan_overflow(c, c->last_buf, c->last_B, ccap))) return rc;
  }
  hipLaunchKernelGGL(k_reset_check, dim3(1), dim3(64), 0, c->stream, ds);
  const unsigned fgrid = (unsigned)std::max(1, c->num_cu) * c->frame_wg;
  hipLaunchKernelGGL(k_frame, dim3(fgrid), dim3(256), 0, c->stream, c->last_buf, c->last_B, c->cpos.as<uint64_t>(),
                     ccap, n, c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift, c->rd.as<RecDesc>(),
                     pf, pf + n, c->slow.as<uint32_t>(), ds, 0);
  // the frames the canonical parser declined (the frame pass decides a call
  // whose chain ends at such a frame: its failure comes first)
  EW_CHECK(c->cat.ensure((size_t)1 << 20));
  hipLaunchKernelGGL(k_decode_slow, dim3(64), dim3(256), 0, c->stream, c->last_buf, c->last_B, c->cpos.as<uint64_t>(),
                     (const uint32_t *)nullptr, c->slow.as<uint32_t>(), ds, c->pwave.as<uint32_t>(),
                     c->v.as<uint32_t>(), tb->slice, tb->shift, c->rd.as<RecDesc>(), pf, pf + n, (uint32_t)n,
                     c->cat.as<uint8_t>(), (uint64_t)c->cat.cap);
  const uint32_t nb = grid_for(n, 1024);
  const size_t had = c->lbstat.cap;
  EW_CHECK(c->lbstat.ensure((size_t)nb * 8));
  c->epoch = (c->epoch + 1) & 0xffffffu;
  if (c->lbstat.cap != had || c->epoch == 0) {
    EW_CHECK(hipMemsetAsync(c->lbstat.p, 0, c->lbstat.cap, c->stream));
    if (c->epoch == 0) c->epoch = 1;
  }
  // k_check's ents / metadata / unknown-field lists go to scratch: the
  // call's ents (ewal_copy_entries) are the frame pass's, with index
  // rewinds already applied (wal/wal.go:173), and must survive this
  EW_CHECK(c->opf.ensure((size_t)nb * 4));
  EW_CHECK(c->rmlist.ensure((size_t)n * 4));
  EW_CHECK(c->rents.ensure((size_t)n * sizeof(ewal_entry)));
  EW_CHECK(c->rulist.ensure((size_t)n * sizeof(uint2)));
  SegArgs useg{};
  useg.ulist = c->rulist.as<uint2>();
  hipLaunchKernelGGL(k_check<false>, dim3(nb), dim3(1024), 0, c->stream, tb->shift, c->rd.as<RecDesc>(), (uint32_t)n,
                     (const uint32_t *)pf, (const uint32_t *)(pf + n), c->last_ri, c->lbstat.as<unsigned long long>(),
                     c->epoch, c->opf.as<uint32_t>(), c->rents.as<ewal_entry>(), c->rmlist.as<uint32_t>(), ds, useg,
                     (const uint32_t *)nullptr);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipStreamSynchronize(c->stream));
  c->rd_valid = true;
  return 0;
}

extern "C" {

int ewal_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ewal_ctx_create(int device, ewal_ctx **out) {
  *out = nullptr;
  int n = ewal_device_count();
  if (n <= 0) return EWAL_E_NODEVICE;
  if (device < 0 || device >= n) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(device));
  auto *c = new ewal_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->num_cu = prop.multiProcessorCount;
  // a blocking stream: ordered with the legacy default stream, so device
  // buffers a caller filled there (torch's default stream, hipMemcpy) are
  // complete before the ctx's kernels read them, and its results before the
  // caller's next default-stream work reads them
  EW_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamDefault));
  c->own_stream = true;
#ifdef EW_ABLATION_HOOKS   // timing experiments only (tools/): results are wrong under ablation.  The product
                           // build reads no environment variable: its path is set by ewal_ctx_set_options only.
  if (const char *e = std::getenv("EWAL_STREAM_ABLATE")) c->ablate = std::atoi(e);
  if (const char *e = std::getenv("EWAL_FRAME_WG")) c->frame_wg = std::max(1, std::min(16, std::atoi(e)));
  if (const char *e = std::getenv("EWAL_OV")) {   // "0": the serial pipeline; "C,F": overlapped, C chunks, F frame CUs
    int ch = 0, fc = 0;
    if (std::sscanf(e, "%d,%d", &ch, &fc) >= 1 && ch <= 0) c->ov_state = -1;
    c->ov_opt = ch > 0;
    if (ch > 0) c->ov_chunks = std::min(ch, 64);
    if (fc > 0) c->ov_fcus = fc;
  }
  if (const char *e = std::getenv("EWAL_OV_NOFR")) c->ov_nofr = std::atoi(e);
#endif
  EW_CHECK(hipEventCreate(&c->ev0));
  EW_CHECK(hipEventCreate(&c->ev1));
  EW_CHECK(hipEventCreate(&c->evs0));
  EW_CHECK(hipEventCreate(&c->evs1));
  EW_CHECK(hipEventCreate(&c->evf0));
  EW_CHECK(hipEventCreate(&c->evf1));
  EW_CHECK(hipHostMalloc((void **)&c->h_small, sizeof(Small), hipHostMallocMapped));
  EW_CHECK(hipHostMalloc((void **)&c->h_res, sizeof(ResultDev), hipHostMallocMapped));
  EW_CHECK(hipHostGetDevicePointer((void **)&c->h_small_dev, c->h_small, 0));
  EW_CHECK(hipHostGetDevicePointer((void **)&c->h_res_dev, c->h_res, 0));
  EW_CHECK(c->small.ensure(sizeof(Small)));
  *out = c;
  return EWAL_OK;
}

void ewal_ctx_destroy(ewal_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (auto &kv : c->tables) {
    (void)hipFree(kv.second.slice);
    (void)hipFree(kv.second.shift);
    (void)hipFree(kv.second.unib);
  }
  if (c->h_small) (void)hipHostFree(c->h_small);
  if (c->h_res) (void)hipHostFree(c->h_res);
  (void)hipEventDestroy(c->ev0);
  (void)hipEventDestroy(c->ev1);
  (void)hipEventDestroy(c->evs0);
  (void)hipEventDestroy(c->evs1);
  (void)hipEventDestroy(c->evf0);
  (void)hipEventDestroy(c->evf1);
  for (hipEvent_t e : c->ov_ev) (void)hipEventDestroy(e);
  ov_unregister(c);
  ov_release_streams(c);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int ewal_ctx_set_stream(ewal_ctx *c, void *s) {
  if (!c) return EWAL_E_INVAL;
  (void)hipSetDevice(c->device);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  if (s) {
    c->stream = (hipStream_t)s;
    c->own_stream = false;
  } else {
    EW_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamDefault));   // blocking, as in ewal_ctx_create
    c->own_stream = true;
  }
  return EWAL_OK;
}

int ewal_ctx_set_options(ewal_ctx *c, uint32_t opts) {
  const uint32_t known = EWAL_OPT_GENERAL_PATH | EWAL_OPT_OVERLAP | EWAL_OPT_VH_ON | EWAL_OPT_VH_OFF;
  if (!c || (opts & ~known) || ((opts & EWAL_OPT_VH_ON) && (opts & EWAL_OPT_VH_OFF))) return EWAL_E_INVAL;
  c->fused = (opts & EWAL_OPT_GENERAL_PATH) ? 0 : 1;
  c->ov_opt = (opts & EWAL_OPT_OVERLAP) != 0;
  c->vh_opt = (opts & EWAL_OPT_VH_ON) ? 1 : (opts & EWAL_OPT_VH_OFF) ? -1 : 0;
  return EWAL_OK;
}

int ewal_ctx_reserve(ewal_ctx *c, uint64_t wal_bytes, uint32_t flags) {
  if (!c) return EWAL_E_INVAL;
  if (flags & EWAL_RESERVE_HOST_STAGING) {   // the HBM copy of host bytes (ewal_readall_host / ewal_wal_readall)
    EW_CHECK(hipSetDevice(c->device));
    EW_CHECK(stage_ensure(c, wal_bytes + 16));
  }
  EW_CHECK(hipSetDevice(c->device));
  DevTables *tb;
  int rc = get_tables(c, 0x82F63B78u, &tb);
  if (rc) return rc;
  const uint64_t B = wal_bytes;
  if ((rc = stream_ensure(c, B, 1))) return rc;
  const uint64_t ccap = cand_cap(B);
  EW_CHECK(c->cpos.ensure(ccap * 8));
  // the fused pass: look-back words, tile records, ents / mlist for the
  // first call's descriptor capacity (readall_impl's rdcap)
  {
    const uint32_t nunits = (uint32_t)(B / EW_WAVE_BYTES + 1);
    const uint32_t tu = 1u << fr_tsh(c, nunits);
    if ((rc = fr_ensure(c, nunits, (nunits + tu - 1) / tu))) return rc;
  }
  const uint64_t ecap = std::min<uint64_t>(ccap, B / 4096 + 1024);
  EW_CHECK(c->ents.ensure((size_t)ecap * sizeof(ewal_entry)));
  EW_CHECK(c->mlist.ensure((size_t)4096 * 8));
  // load the device code: a ReadAll over a one-frame WAL (a crcType record)
  static const uint8_t tiny[16] = {4, 0, 0, 0, 0, 0, 0, 0, 0x08, 0x04, 0x10, 0x00};
  EW_CHECK(stage_ensure(c, 64));
  EW_CHECK(hipMemcpyAsync(c->hbuf_dev.p, tiny, sizeof(tiny), hipMemcpyHostToDevice, c->stream));
  ewal_result r;
  rc = readall_impl(c, c->hbuf_dev.as<uint8_t>(), 12, 0, &r);
  c->last_k = 0;
  EW_CHECK(hipStreamSynchronize(c->stream));
  return rc < 0 ? rc : EWAL_OK;
}

int ewal_readall_device(ewal_ctx *c, const void *d_buf, uint64_t len, uint64_t ri, ewal_result *out) {
  if (!c || !out || (!d_buf && len)) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  return readall_impl(c, (const uint8_t *)d_buf, len, ri, out);
}

int ewal_readall_range_device(ewal_ctx *c, const void *d_buf, uint64_t len, uint64_t ri, uint32_t flags,
                              ewal_result *out) {
  if (!c || !out || (!d_buf && len) || (flags & ~(uint32_t)EWAL_RANGE_DEFER_FIRST)) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  c->defer_first = (flags & EWAL_RANGE_DEFER_FIRST) != 0;
  const int rc = readall_impl(c, (const uint8_t *)d_buf, len, ri, out);
  c->defer_first = false;
  return rc;
}

int ewal_range_probe(ewal_ctx *c, const void *d_buf, uint64_t len, uint64_t from, uint64_t window, int64_t *pos,
                     int64_t *first_entry_index) {
  return ewal_range_probe_aligned(c, d_buf, len, from, window, 1, pos, first_entry_index);
}

int ewal_range_probe_aligned(ewal_ctx *c, const void *d_buf, uint64_t len, uint64_t from, uint64_t window,
                             uint32_t align, int64_t *pos, int64_t *first_entry_index) {
  if (!c || !pos || !first_entry_index || (!d_buf && len) || !align || (align & (align - 1))) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  *pos = -1;
  *first_entry_index = -1;
  if (from >= len) return EWAL_OK;
  const uint64_t end = std::min<uint64_t>(len, from + std::max<uint64_t>(window, 1));
  EW_CHECK(c->sdesc.ensure(32));
  unsigned long long *dpos = c->sdesc.as<unsigned long long>();
  long long *dout = (long long *)(dpos + 1);
  EW_CHECK(hipMemsetAsync(dpos, 0xff, 8, c->stream));
  const unsigned grid = (unsigned)std::min<uint64_t>(grid_for(end - from, 256), (uint64_t)std::max(1, c->num_cu) * 8);
  hipLaunchKernelGGL(k_probe_cand, dim3(grid), dim3(256), 0, c->stream, (const uint8_t *)d_buf, len, from, end, align,
                     dpos);
  hipLaunchKernelGGL(k_probe_walk, dim3(1), dim3(64), 0, c->stream, (const uint8_t *)d_buf, len,
                     (const unsigned long long *)dpos, 64u, dout);
  EW_CHECK(hipGetLastError());
  long long h[2];
  EW_CHECK(hipMemcpyAsync(h, dout, 16, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  *pos = h[0];
  *first_entry_index = h[1];
  return EWAL_OK;
}

int ewal_readall_batch_device(ewal_ctx *c, const void *d_buf, uint64_t n_shards, const uint64_t *lens,
                              const uint64_t *ri, ewal_result *out) {
  if (!c || (n_shards && (!lens || !ri || !out)) || n_shards >= 0x7fffffffull) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  return readall_batch_impl(c, (const uint8_t *)d_buf, (uint32_t)n_shards, lens, ri, out);
}

int64_t ewal_batch_copy_entries(ewal_ctx *c, uint64_t shard, ewal_entry *out, int64_t cap) {
  if (!c || (!out && cap) || shard >= c->bnents.size()) return EWAL_E_INVAL;
  const int64_t n = std::min<int64_t>(cap, (int64_t)c->bnents[shard]);
  if (n > 0) {
    EW_CHECK(hipMemcpyAsync(out, c->bents.as<ewal_entry>() + c->bent_first[shard], (size_t)n * sizeof(ewal_entry),
                            hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
  }
  return n;
}

int64_t ewal_batch_copy_unrec(ewal_ctx *c, uint64_t shard, ewal_unrec *out, int64_t cap) {
  if (!c || (!out && cap) || shard >= c->bunrec.size()) return EWAL_E_INVAL;
  const std::vector<ewal_unrec> &u = c->bunrec[shard];
  const int64_t n = std::min<int64_t>(cap, (int64_t)u.size());
  if (n > 0) std::memcpy(out, u.data(), (size_t)n * sizeof(ewal_unrec));
  return n;
}

int64_t ewal_batch_copy_unrec_bytes(ewal_ctx *c, uint64_t shard, uint8_t *out, int64_t cap) {
  if (!c || (!out && cap) || shard >= c->bunrec_bytes.size()) return EWAL_E_INVAL;
  const std::vector<uint8_t> &b = c->bunrec_bytes[shard];
  const int64_t n = std::min<int64_t>(cap, (int64_t)b.size());
  if (n > 0) std::memcpy(out, b.data(), (size_t)n);
  return n;
}

int ewal_device_alloc(ewal_ctx *c, uint64_t len, void **d_out) {
  if (!c || !d_out) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  if (hipMalloc(d_out, std::max<uint64_t>(len, 16)) != hipSuccess) return EWAL_E_NOMEM;
  return EWAL_OK;
}
int ewal_device_free(ewal_ctx *c, void *d) {
  if (!c) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  if (d) EW_CHECK(hipFree(d));
  return EWAL_OK;
}
int ewal_upload(ewal_ctx *c, void *d, const void *h, uint64_t len) {
  if (!c || (len && (!d || !h))) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  if (len) EW_CHECK(hipMemcpyAsync(d, h, len, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  return EWAL_OK;
}
int ewal_download(ewal_ctx *c, void *h, const void *d, uint64_t len) {
  if (!c || (len && (!d || !h))) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  if (len) EW_CHECK(hipMemcpyAsync(h, d, len, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  return EWAL_OK;
}

int ewal_stage_to_device(ewal_ctx *c, const void *h_buf, uint64_t len, void **d_out) {
  if (!c || !d_out || (!h_buf && len)) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  EW_CHECK(stage_ensure(c, len + 16));
  if (len) EW_CHECK(hipMemcpyAsync(c->hbuf_dev.p, h_buf, len, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  *d_out = c->hbuf_dev.p;
  return EWAL_OK;
}

int ewal_stage_begin(ewal_ctx *c, uint64_t len) {
  if (!c) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  EW_CHECK(stage_ensure(c, len + 16));
  return EWAL_OK;
}
int ewal_stage_put(ewal_ctx *c, uint64_t off, const void *h, uint64_t n) {
  if (!c || (n && !h) || off + n + 16 > c->hbuf_dev.cap) return EWAL_E_INVAL;
  if (n) EW_CHECK(hipMemcpyAsync(c->hbuf_dev.as<uint8_t>() + off, h, n, hipMemcpyHostToDevice, c->stream));
  return EWAL_OK;
}
int ewal_stage_sync(ewal_ctx *c) {
  if (!c) return EWAL_E_INVAL;
  EW_CHECK(hipStreamSynchronize(c->stream));
  return EWAL_OK;
}
int ewal_stage_readall(ewal_ctx *c, uint64_t len, uint64_t ri, ewal_result *out) {
  if (!c || !out || len + 16 > c->hbuf_dev.cap) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  return readall_impl(c, c->hbuf_dev.as<uint8_t>(), len, ri, out);
}

int ewal_readall_host(ewal_ctx *c, const void *h_buf, uint64_t len, uint64_t ri, ewal_result *out) {
  if (!c || !out || (!h_buf && len)) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  EW_CHECK(stage_ensure(c, len + 16));
  if (len) EW_CHECK(hipMemcpyAsync(c->hbuf_dev.p, h_buf, len, hipMemcpyHostToDevice, c->stream));
  return readall_impl(c, c->hbuf_dev.as<uint8_t>(), len, ri, out);
}

int64_t ewal_copy_entries(ewal_ctx *c, ewal_entry *out, int64_t cap) {
  if (!c || (!out && cap)) return EWAL_E_INVAL;
  if (!c->last_ok) return 0;
  int64_t n = std::min<int64_t>(cap, (int64_t)c->last_nents);
  if (n > 0) {
    EW_CHECK(hipMemcpyAsync(out, c->ents.p, (size_t)n * sizeof(ewal_entry), hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
  }
  return n;
}

int64_t ewal_copy_unrec(ewal_ctx *c, ewal_unrec *out, int64_t cap) {
  if (!c || (!out && cap)) return EWAL_E_INVAL;
  if (!c->last_ok) return 0;
  const int64_t n = std::min<int64_t>(cap, (int64_t)c->unrec.size());
  if (n > 0) std::memcpy(out, c->unrec.data(), (size_t)n * sizeof(ewal_unrec));
  return n;
}

int64_t ewal_copy_unrec_bytes(ewal_ctx *c, uint8_t *out, int64_t cap) {
  if (!c || (!out && cap)) return EWAL_E_INVAL;
  if (!c->last_ok) return 0;
  const int64_t n = std::min<int64_t>(cap, (int64_t)c->unrec_bytes);
  if (n > 0) {
    EW_CHECK(hipSetDevice(c->device));
    EW_CHECK(hipMemcpy(out, c->uarena.p, (size_t)n, hipMemcpyDeviceToHost));
  }
  return n;
}

int64_t ewal_copy_split_bytes(ewal_ctx *c, uint8_t *out, int64_t cap) {
  if (!c || (!out && cap) || cap < 0) return EWAL_E_INVAL;
  const int64_t n = std::min<int64_t>(cap, (int64_t)c->cat_bytes);
  if (n > 0) {
    EW_CHECK(hipSetDevice(c->device));
    EW_CHECK(hipMemcpy(out, c->cat.p, (size_t)n, hipMemcpyDeviceToHost));
  }
  return (int64_t)c->cat_bytes;
}

int64_t ewal_batch_copy_split_bytes(ewal_ctx *c, uint64_t shard, uint8_t *out, int64_t cap) {
  if (!c || (!out && cap) || cap < 0 || shard >= c->bsplit_bytes.size()) return EWAL_E_INVAL;
  const std::vector<uint8_t> &b = c->bsplit_bytes[shard];
  const int64_t n = std::min<int64_t>(cap, (int64_t)b.size());
  if (n > 0) std::memcpy(out, b.data(), (size_t)n);
  return (int64_t)b.size();
}

// The last ReadAll's per-frame descriptors in c->rd (rebuilt when the fused
// pass decided it); EWAL_E_INVAL when another call took the state they come from.
static int need_records(ewal_ctx *c) {
  if (!c->rec_valid) return EWAL_E_INVAL;
  if (c->last_n && !c->rd_valid) {   // the fused pass kept no descriptors: decode them now
    if (!c->rec_rebuild) return EWAL_E_INVAL;
    EW_CHECK(hipSetDevice(c->device));
    return materialise_records(c);
  }
  return 0;
}

int64_t ewal_copy_records(ewal_ctx *c, ewal_record *out, int64_t cap) {
  if (!c || (!out && cap) || !c->rec_valid) return EWAL_E_INVAL;
  int64_t n = std::min<int64_t>(cap, (int64_t)c->last_n);
  if (n > 0) {
    if (int rc = need_records(c)) return rc;
  }
  if (n > 0) {
    EW_CHECK(c->recs.ensure((size_t)n * sizeof(ewal_record)));
    hipLaunchKernelGGL(k_records_out, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, c->rd.as<RecDesc>(),
                       (uint32_t)n, c->recs.as<ewal_record>());
    EW_CHECK(hipMemcpyAsync(out, c->recs.p, (size_t)n * sizeof(ewal_record), hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
  }
  return n;
}

// The range info of a ReadAll the frame pass decided, from its reductions
// (k_range_info_fr): the fields k_range_info derives from the descriptors.
// 1: an entry below ri or an index rewind was met (the descriptors decide).
static int range_info_fused(ewal_ctx *c, ewal_range_info &o) {
  const Small &hs = c->fi_small;
  if (hs.fr_below || (c->fi_a.rew && hs.fr_rews)) return 1;
  EW_CHECK(hipSetDevice(c->device));
  EW_CHECK(c->rfr.ensure(sizeof(RangeFr)));
  RangeFr *d = c->rfr.as<RangeFr>();
  const FrArgs &a = c->fi_a;
  const uint64_t K = c->last_n;
#define RFR_LAUNCH(T) hipLaunchKernelGGL(k_range_info_fr<T>, dim3(1), dim3(512), 0, c->stream, a, hs.nmeta, \
                                         hs.fc.meta_inv, hs.fr.le, hs.fr.lo, hs.fr.ls, (unsigned long long)K, d)
  if (c->fi_tsh == 8) RFR_LAUNCH(8);
  else if (c->fi_tsh == 6) RFR_LAUNCH(6);
  else RFR_LAUNCH(4);
#undef RFR_LAUNCH
  EW_CHECK(hipGetLastError());
  RangeFr h;
  EW_CHECK(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  const RecDesc &f = h.d[6];   // frame 0 (fused: its canonical fields; no failure before the CRC check)
  o.first_type = f.type;
  if (f.type == 4) o.first_crc = f.crc;
  o.first_dlen = f.dlen;
  o.first_stored_crc = f.crc;
  o.first_u0 = f.type == 4 ? f.crc : h.u0;
  o.first_pre_crc = 0;
  if (h.pos[0] != ~0ull) {
    o.md_first_frame = (int64_t)h.ord[0];
    if (!h.d[0].dnil && h.d[0].dlen) {
      o.md_first_off = (int64_t)h.d[0].doff;
      o.md_first_len = (int64_t)h.d[0].dlen;
    }
  }
  if (h.pos[1] != ~0ull) {
    o.md_value_frame = (int64_t)h.ord[1];
    o.md_value_off = (int64_t)h.d[1].doff;
    o.md_value_len = (int64_t)h.d[1].dlen;
  }
  if (h.pos[2] != ~0ull && h.pos[3] != ~0ull) {
    o.first_entry_frame = (int64_t)h.ord[2];
    o.first_entry_index = h.d[2].f1;
    o.min_entry_index = h.d[2].f1;   // no entry below ri, ops in order: the first op's
    o.last_entry_frame = (int64_t)h.ord[3];
    o.last_entry_index = h.d[3].f1;
    if (h.pos[4] != ~0ull) {
      o.last_op_frame = (int64_t)h.ord[4];
      o.last_op_index = h.d[4].f1;
    }
  }
  if (h.pos[5] != ~0ull) {
    o.state_frame = (int64_t)h.ord[5];
    o.state_term = h.d[5].f0;
    o.state_vote = h.d[5].f1;
    o.state_commit = h.d[5].f2;
  }
  return 0;
}

int ewal_copy_range_info(ewal_ctx *c, ewal_range_info *out) {
  if (!c || !out) return EWAL_E_INVAL;
  ewal_range_info o;
  std::memset(&o, 0, sizeof(o));
  o.first_crc = o.md_first_frame = o.md_value_frame = o.first_entry_frame = o.last_entry_frame = -1;
  o.last_op_frame = -1;
  o.md_first_off = o.md_value_off = -1;
  o.first_type = -1;
  o.state_frame = -1;
  if (!c->rec_valid) return EWAL_E_INVAL;
  const uint64_t n = c->last_n;
  o.n_frames = (int64_t)n;
  o.end_off = c->last_q;
  o.n_bytes = c->last_B;
  if (n && !c->rd_valid && c->rec_rebuild && c->fi_valid) {
    const int rc = range_info_fused(c, o);
    if (rc < 0) return rc;
    if (rc == 0) {
      *out = o;
      return EWAL_OK;
    }
  }
  if (int rc = need_records(c)) return rc;
  if (n) {
    EW_CHECK(c->sdesc.ensure(sizeof(RangeDev)));
    RangeDev h0{~0ull, ~0ull, ~0ull, ~0ull, 0ull, 0ull, 0ull}, h;
    EW_CHECK(hipMemcpyAsync(c->sdesc.p, &h0, sizeof(h0), hipMemcpyHostToDevice, c->stream));
    const RecDesc *rd = c->rd.as<RecDesc>();
    hipLaunchKernelGGL(k_range_info, dim3((unsigned)std::min<uint64_t>(grid_for(n, 256), 1024)), dim3(256), 0,
                       c->stream, rd, (uint32_t)n, c->last_ri, c->sdesc.as<RangeDev>());
    EW_CHECK(hipGetLastError());
    EW_CHECK(hipMemcpyAsync(&h, c->sdesc.p, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
    auto frame = [&](uint64_t r, RecDesc *d) {
      return hipMemcpy(d, rd + r, sizeof(RecDesc), hipMemcpyDeviceToHost);
    };
    RecDesc d;
    EW_CHECK(frame(0, &d));
    if (d.type == 4) o.first_crc = d.crc;
    o.first_type = d.type;
    o.first_dlen = d.dlen;
    o.first_stored_crc = d.crc;
    o.first_u0 = d.chained;   // k_check ran frame 0 from seed 0: crc32.Update(0, Data) (crcType: the stored CRC)
    {   // k_check left the frame's verdict in d.st: framing / Record.Unmarshal fail before decoder.decode's
        // Validate; the Entry / HardState decode (sub_st), ReadAll's type / metadata / gap rules after it
      const bool post = d.st == EWAL_ERR_RECORD_CRC || d.st == EWAL_ERR_WAL_CRC || d.st == EWAL_ERR_UNEXPECTED_TYPE ||
                        d.st == EWAL_ERR_METADATA_CONFLICT || d.st == EWAL_PANIC_INDEX_GAP || d.sub_st != 0;
      o.first_pre_crc = d.st != 0 && !post;
    }
    if (h.md_first != ~0ull) {
      EW_CHECK(frame(h.md_first, &d));
      o.md_first_frame = (int64_t)h.md_first;
      if (!d.dnil && d.dlen) {
        o.md_first_off = (int64_t)(d.pad0 == 2 ? rd_cat_off(d) : d.doff);
        o.md_first_len = (int64_t)d.dlen;
        if (d.pad0 == 2) o.md_split |= 1;
      }
    }
    if (h.md_value != ~0ull) {
      EW_CHECK(frame(h.md_value, &d));
      o.md_value_frame = (int64_t)h.md_value;
      o.md_value_off = (int64_t)(d.pad0 == 2 ? rd_cat_off(d) : d.doff);
      o.md_value_len = (int64_t)d.dlen;
      if (d.pad0 == 2) o.md_split |= 2;
    }
    if (h.ent_first != ~0ull) {
      EW_CHECK(frame(h.ent_first, &d));
      o.first_entry_frame = (int64_t)h.ent_first;
      o.first_entry_index = d.f1;
      o.min_entry_index = h.min_index;
      EW_CHECK(frame(h.ent_last1 - 1, &d));
      o.last_entry_frame = (int64_t)(h.ent_last1 - 1);
      o.last_entry_index = d.f1;
      if (h.op_last1) {
        EW_CHECK(frame(h.op_last1 - 1, &d));
        o.last_op_frame = (int64_t)(h.op_last1 - 1);
        o.last_op_index = d.f1;
      }
    }
    if (h.st_last1) {   // the range's HardState (its last stateType frame)
      EW_CHECK(frame(h.st_last1 - 1, &d));
      o.state_frame = (int64_t)(h.st_last1 - 1);
      o.state_term = d.f0;
      o.state_vote = d.f1;
      o.state_commit = d.f2;
      o.state_unrec = d.pad1 & 1;
    }
  }
  *out = o;
  return EWAL_OK;
}

int ewal_encode_entries_device(ewal_ctx *c, const void *d_data, uint64_t data_len_total, const ewal_entry *d_ents,
                               uint64_t n, uint32_t prev_crc, void *d_out, uint64_t cap, uint64_t *out_len,
                               uint32_t *last_crc) {
  if (!c || !out_len || !last_crc || (n && (!d_ents || !d_out)) || (data_len_total && !d_data)) return EWAL_E_INVAL;
  *out_len = 0;
  *last_crc = prev_crc;
  if (n == 0) return EWAL_OK;
  if (n >= 0x7fffffffull) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  DevTables *tb;
  int rc = get_tables(c, 0x82F63B78u, &tb);
  if (rc) return rc;
  EW_CHECK(c->small.ensure(sizeof(Small)));
  Small *ds = c->small.as<Small>();
  EW_CHECK(hipMemsetAsync(&ds->errflag, 0, 4, c->stream));
  // per-entry scratch: esz, xoff, fsz, foff (u64) + crc (u32)
  EW_CHECK(c->encw.ensure((size_t)n * 36 + 64));
  uint64_t *esz = c->encw.as<uint64_t>(), *xoff = esz + n, *fsz = xoff + n, *foff = fsz + n;
  uint32_t *crc = (uint32_t *)(foff + n);
  hipLaunchKernelGGL(k_enc_sizes, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, d_ents, n, data_len_total, esz,
                     &ds->errflag);
  size_t tbytes = 0;
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, esz, xoff, (int)n, c->stream));
  EW_CHECK(c->tmp.ensure(tbytes));
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, tbytes, esz, xoff, (int)n, c->stream));
  uint64_t tail[2];
  uint32_t bad = 0;
  EW_CHECK(hipMemcpyAsync(&tail[0], xoff + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[1], esz + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&bad, &ds->errflag, 4, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  if (bad) return EWAL_E_INVAL;
  const uint64_t E = tail[0] + tail[1];                 // bytes of the data-only stream
  EW_CHECK(c->encs.ensure(E + 64));
  uint8_t *es = c->encs.as<uint8_t>();
  const unsigned wgrid = (unsigned)std::min<uint64_t>(grid_for(n, 4), (uint64_t)c->num_cu * 8);
  hipLaunchKernelGGL(k_enc_body, dim3(wgrid), dim3(256), 0, c->stream, (const uint8_t *)d_data, data_len_total,
                     d_ents, n, xoff, es);
  hipLaunchKernelGGL(k_enc_xor4, dim3(1), dim3(64), 0, c->stream, es, ~prev_crc);
  rc = run_stream(c, tb, es, E, 0, 0);
  if (rc) return rc;
  hipLaunchKernelGGL(k_enc_crc, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, es, xoff, esz, n,
                     c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift, crc, fsz);
  hipLaunchKernelGGL(k_enc_xor4, dim3(1), dim3(64), 0, c->stream, es, ~prev_crc);   // the bytes back
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, fsz, foff, (int)n, c->stream));
  EW_CHECK(c->tmp.ensure(tbytes));
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, tbytes, fsz, foff, (int)n, c->stream));
  uint32_t lc = 0;
  EW_CHECK(hipMemcpyAsync(&tail[0], foff + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[1], fsz + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&lc, crc + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  const uint64_t total = tail[0] + tail[1];
  if (total > cap) return EWAL_E_NOMEM;
  hipLaunchKernelGGL(k_enc_frame, dim3(wgrid), dim3(256), 0, c->stream, es, E, xoff, esz, crc, foff, n,
                     (uint8_t *)d_out);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipStreamSynchronize(c->stream));
  *out_len = total;
  *last_crc = lc;
  return EWAL_OK;
}

int ewal_save_device(ewal_ctx *c, const void *d_data, uint64_t data_len_total, const ewal_save_rec *d_recs, uint64_t n,
                     uint32_t prev_crc, void *d_out, uint64_t cap, uint64_t *out_len, uint32_t *last_crc,
                     uint64_t *h_rec_off) {
  if (!c || !out_len || !last_crc || (n && (!d_recs || !d_out)) || (data_len_total && !d_data)) return EWAL_E_INVAL;
  *out_len = 0;
  *last_crc = prev_crc;
  if (n == 0) return EWAL_OK;
  if (n >= 0x7fffffffull) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  DevTables *tb;
  int rc = get_tables(c, 0x82F63B78u, &tb);
  if (rc) return rc;
  EW_CHECK(c->small.ensure(sizeof(Small)));
  Small *ds = c->small.as<Small>();
  EW_CHECK(hipMemsetAsync(&ds->errflag, 0, 4, c->stream));
  // per-record scratch: esz, xoff, fsz, foff (u64) + crc, pcrc (u32)
  EW_CHECK(c->encw.ensure((size_t)n * 40 + 64));
  uint64_t *esz = c->encw.as<uint64_t>(), *xoff = esz + n, *fsz = xoff + n, *foff = fsz + n;
  uint32_t *crc = (uint32_t *)(foff + n), *pcrc = crc + n;
  hipLaunchKernelGGL(k_save_sizes, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, d_recs, n, data_len_total, esz,
                     &ds->errflag);
  size_t tbytes = 0;
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, esz, xoff, (int)n, c->stream));
  EW_CHECK(c->tmp.ensure(tbytes));
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, tbytes, esz, xoff, (int)n, c->stream));
  uint64_t tail[2];
  uint32_t bad = 0;
  EW_CHECK(hipMemcpyAsync(&tail[0], xoff + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[1], esz + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&bad, &ds->errflag, 4, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  if (bad) return EWAL_E_INVAL;
  const uint64_t E = tail[0] + tail[1];                 // bytes of the data-only stream
  EW_CHECK(c->encs.ensure(E + 64));
  uint8_t *es = c->encs.as<uint8_t>();
  const unsigned wgrid = (unsigned)std::min<uint64_t>(grid_for(n, 4), (uint64_t)c->num_cu * 8);
  const uint32_t R0 = ~prev_crc;
  hipLaunchKernelGGL(k_save_body, dim3(wgrid), dim3(256), 0, c->stream, (const uint8_t *)d_data, data_len_total,
                     d_recs, n, xoff, es);
  if (E) {
    hipLaunchKernelGGL(k_save_xor4, dim3(1), dim3(64), 0, c->stream, es, E, R0);
    rc = run_stream(c, tb, es, E, 0, 0);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_save_crc, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, es, E, d_recs, xoff, esz, n, R0,
                     c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift, crc, pcrc, fsz);
  if (E) hipLaunchKernelGGL(k_save_xor4, dim3(1), dim3(64), 0, c->stream, es, E, R0);   // the bytes back
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, fsz, foff, (int)n, c->stream));
  EW_CHECK(c->tmp.ensure(tbytes));
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, tbytes, fsz, foff, (int)n, c->stream));
  uint32_t lc = 0;
  EW_CHECK(hipMemcpyAsync(&tail[0], foff + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[1], fsz + n - 1, 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&lc, crc + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
  if (h_rec_off) EW_CHECK(hipMemcpyAsync(h_rec_off, foff, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  const uint64_t total = tail[0] + tail[1];
  if (total > cap) return EWAL_E_NOMEM;
  hipLaunchKernelGGL(k_save_frame, dim3(wgrid), dim3(256), 0, c->stream, es, E, d_recs, xoff, esz, crc, pcrc, foff, n,
                     (uint8_t *)d_out);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipStreamSynchronize(c->stream));
  *out_len = total;
  *last_crc = lc;
  return EWAL_OK;
}

int ewal_crc32_update_device(ewal_ctx *c, uint32_t crc, uint32_t poly, const void *d_buf, uint64_t n, uint32_t *out) {
  if (!c || !out || (!d_buf && n)) return EWAL_E_INVAL;
  if (n == 0) { *out = crc; return EWAL_OK; }
  if (((uintptr_t)d_buf & 15) != 0) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  DevTables *tb;
  int rc = get_tables(c, poly, &tb);
  if (rc) return rc;
  EW_CHECK(c->small.ensure(sizeof(Small)));
  rc = run_stream(c, tb, (const uint8_t *)d_buf, n, 0, 0);
  if (rc) return rc;
  // P(n) = lin(all n bytes) from the stream prefixes (one thread).
  EW_CHECK(c->sdesc.ensure(sizeof(uint32_t)));
  hipLaunchKernelGGL(k_prefix_one, dim3(1), dim3(64), 0, c->stream, (const uint8_t *)d_buf, c->pwave.as<uint32_t>(),
                     c->v.as<uint32_t>(), tb->slice, tb->shift, n, c->sdesc.as<uint32_t>());
  uint32_t P = 0;
  EW_CHECK(hipMemcpyAsync(&P, c->sdesc.p, 4, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  const ewal::CrcTables &ht = *c->host_tables[poly];
  // Update(crc, D) = S_n(crc ^ ~0) ^ lin(D) ^ ~0
  *out = ht.shift_n(n, crc ^ 0xffffffffu) ^ P ^ 0xffffffffu;
  return EWAL_OK;
}

// The files k_snap left to the residual decode (h[i].resid): gather split
// envelope Data, count and place the segments, decode.  Rare: the extents
// come back to the host between the steps.
static int snap_residuals(ewal_ctx *c, const uint8_t *buf, uint32_t n, SnapDesc *h) {
  c->snap_buf = buf;
  c->snap_n = n;
  c->snap_rmap.assign(n, -1);
  c->snap_rfirst.clear();
  c->snap_rcnt.clear();
  std::vector<uint32_t> rl;
  std::vector<uint64_t> goff;
  uint64_t gtot = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (h[i].st != EWAL_OK || !h[i].resid) continue;
    c->snap_rmap[i] = (int32_t)rl.size();
    rl.push_back(i);
    goff.push_back(gtot);
    if (h[i].resid == 2) gtot += h[i].dlen;
  }
  const uint32_t nr = (uint32_t)rl.size();
  if (!nr) return EWAL_OK;
  EW_CHECK(c->srlist.ensure((size_t)nr * 4));
  EW_CHECK(c->sgoff.ensure((size_t)nr * 8));
  EW_CHECK(c->srcnt.ensure((size_t)nr * 8));
  EW_CHECK(c->srfirst.ensure((size_t)nr * 8));
  EW_CHECK(c->sgather.ensure((size_t)std::max<uint64_t>(gtot, 1)));
  EW_CHECK(hipMemcpyAsync(c->srlist.p, rl.data(), (size_t)nr * 4, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipMemcpyAsync(c->sgoff.p, goff.data(), (size_t)nr * 8, hipMemcpyHostToDevice, c->stream));
  SnapDesc *sd = c->hsdesc.dev<SnapDesc>();
  esnap_snapshot *snaps = c->snaps.as<esnap_snapshot>();
  if (gtot)
    hipLaunchKernelGGL(k_snap_gather, dim3(nr), dim3(256), 0, c->stream, buf, (const SnapDesc *)sd,
                       c->srlist.as<uint32_t>(), c->sgoff.as<uint64_t>(), c->sgather.as<uint8_t>(), nr);
  hipLaunchKernelGGL(k_snap_resid<false>, dim3(grid_for(nr, 256)), dim3(256), 0, c->stream, buf,
                     (const uint8_t *)c->sgather.as<uint8_t>(), sd, c->srlist.as<uint32_t>(), c->sgoff.as<uint64_t>(), nr,
                     c->srcnt.as<uint64_t>(), (const uint64_t *)nullptr, (emsg_segment *)nullptr, snaps);
  EW_CHECK(hipGetLastError());
  c->snap_rcnt.resize(nr);
  EW_CHECK(hipMemcpyAsync(c->snap_rcnt.data(), c->srcnt.p, (size_t)nr * 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  c->snap_rfirst.resize(nr);
  uint64_t tot = 0;
  for (uint32_t r = 0; r < nr; ++r) {
    c->snap_rfirst[r] = tot;
    tot += c->snap_rcnt[r];
  }
  EW_CHECK(c->ssegs.ensure((size_t)std::max<uint64_t>(tot, 1) * sizeof(emsg_segment)));
  EW_CHECK(hipMemcpyAsync(c->srfirst.p, c->snap_rfirst.data(), (size_t)nr * 8, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_snap_resid<true>, dim3(grid_for(nr, 256)), dim3(256), 0, c->stream, buf,
                     (const uint8_t *)c->sgather.as<uint8_t>(), sd, c->srlist.as<uint32_t>(), c->sgoff.as<uint64_t>(), nr,
                     (uint64_t *)nullptr, (const uint64_t *)c->srfirst.as<uint64_t>(), c->ssegs.as<emsg_segment>(),
                     snaps);
  EW_CHECK(hipGetLastError());
  return EWAL_OK;
}

int esnap_verify_packed(ewal_ctx *c, const void *d_buf, uint64_t buf_len, const uint64_t *offs, const uint64_t *lens,
                        uint32_t n, uint32_t poly, int32_t *status, uint32_t *stored_crc, uint32_t *computed_crc) {
  if (!c || (!d_buf && buf_len) || (n && (!offs || !lens || !status))) return EWAL_E_INVAL;
  if (((uintptr_t)d_buf & 15) != 0) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  for (uint32_t i = 0; i < n; ++i)
    if (offs[i] + lens[i] > buf_len || offs[i] + lens[i] < offs[i]) return EWAL_E_INVAL;
  DevTables *tb;
  int rc = get_tables(c, poly, &tb);
  if (rc) return rc;
  EW_CHECK(c->small.ensure(sizeof(Small)));
  EW_CHECK(hipEventRecord(c->ev0, c->stream));
  if (buf_len) {
    rc = run_stream(c, tb, (const uint8_t *)d_buf, buf_len, 0, 0);
    if (rc) return rc;
  }
  // the per-file table lives in host-mapped pinned memory: k_snap reads the
  // extents and writes the verdicts in place
  EW_CHECK(c->hsdesc.ensure((size_t)std::max<uint32_t>(n, 1) * sizeof(SnapDesc)));
  SnapDesc *h = c->hsdesc.host<SnapDesc>();
  for (uint32_t i = 0; i < n; ++i) {
    std::memset(&h[i], 0, sizeof(SnapDesc));
    h[i].off = offs[i];
    h[i].len = lens[i];
  }
  if (n) {
    EW_CHECK(c->snaps.ensure((size_t)n * sizeof(esnap_snapshot)));
    hipLaunchKernelGGL(k_snap, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, (const uint8_t *)d_buf,
                       c->pwave.as<uint32_t>(), c->v.as<uint32_t>(), tb->slice, tb->shift, c->hsdesc.dev<SnapDesc>(),
                       c->snaps.as<esnap_snapshot>(), n);
    EW_CHECK(hipGetLastError());
  }
  EW_CHECK(hipStreamSynchronize(c->stream));
  rc = snap_residuals(c, (const uint8_t *)d_buf, n, h);
  if (rc) return rc;
  EW_CHECK(hipEventRecord(c->ev1, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < n; ++i) {
    status[i] = h[i].st;
    if (stored_crc) stored_crc[i] = h[i].stored;
    if (computed_crc) computed_crc[i] = h[i].computed;
  }
  return EWAL_OK;
}

int esnap_copy_snapshot(ewal_ctx *c, uint32_t i, esnap_snapshot *out) {
  if (!c || !out) return EWAL_E_INVAL;
  EW_CHECK(hipMemcpy(out, c->snaps.as<esnap_snapshot>() + i, sizeof(*out), hipMemcpyDeviceToHost));
  return EWAL_OK;
}

int64_t esnap_copy_field(ewal_ctx *c, uint32_t i, int32_t field, void *out, int64_t cap) {
  if (!c || i >= c->snap_n || cap < 0 || (!out && cap) || field < ESNAP_FIELD_DATA || field > ESNAP_FIELD_REMOVED)
    return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  esnap_snapshot s;
  EW_CHECK(hipMemcpy(&s, c->snaps.as<esnap_snapshot>() + i, sizeof(s), hipMemcpyDeviceToHost));
  const int32_t r = c->snap_rmap[i];
  std::vector<emsg_segment> sg;
  if (r >= 0 && c->snap_rcnt[r]) {
    sg.resize(c->snap_rcnt[r]);
    EW_CHECK(hipMemcpy(sg.data(), c->ssegs.as<emsg_segment>() + c->snap_rfirst[r], sg.size() * sizeof(emsg_segment),
                       hipMemcpyDeviceToHost));
  }
  uint8_t *ob = (uint8_t *)out;
  uint64_t *ov = (uint64_t *)out;
  if (field == ESNAP_FIELD_NODES || field == ESNAP_FIELD_REMOVED) {
    const bool nodes = field == ESNAP_FIELD_NODES;
    const int64_t total = nodes ? s.n_nodes : s.n_removed;
    if (total <= 64) {
      const int64_t k = std::min(cap, total);
      if (k > 0) std::memcpy(ov, nodes ? s.nodes : s.removed, (size_t)k * 8);
      return total;
    }
    int64_t k = 0;
    const int32_t kind = nodes ? EMSG_SEG_SNAP_NODE : EMSG_SEG_SNAP_REMOVED;
    for (auto &g : sg)
      if (g.kind == kind && k < cap) ov[k++] = g.off;
    return total;
  }
  if (r < 0) {   // the common layout: Data is one range of the file, no XXX_unrecognized
    if (field == ESNAP_FIELD_UNREC) return 0;
    const int64_t k = std::min<int64_t>(cap, (int64_t)s.data_len);
    if (k > 0) EW_CHECK(hipMemcpy(ob, c->snap_buf + s.data_off, (size_t)k, hipMemcpyDeviceToHost));
    return (int64_t)s.data_len;
  }
  const int32_t kind = field == ESNAP_FIELD_DATA ? EMSG_SEG_SNAP_DATA : EMSG_SEG_SNAP_UNREC;
  int64_t total = 0;
  for (auto &g : sg) {
    if (g.kind != kind) continue;
    const int64_t k = std::min<int64_t>(std::max<int64_t>(cap - total, 0), (int64_t)g.len);
    const uint8_t *src = (g.pad ? c->sgather.as<uint8_t>() : c->snap_buf) + g.off;
    if (k > 0) EW_CHECK(hipMemcpy(ob + total, src, (size_t)k, hipMemcpyDeviceToHost));
    total += (int64_t)g.len;
  }
  return total;
}

int emsg_decode_batch_device(ewal_ctx *c, const void *d_buf, uint64_t buf_len, const uint64_t *offs,
                             const uint64_t *lens, uint32_t n, emsg_message *out, uint64_t *n_entries) {
  if (!c || (!d_buf && buf_len) || (n && (!offs || !lens || !out))) return EWAL_E_INVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (offs[i] + lens[i] > buf_len || offs[i] + lens[i] < offs[i] || lens[i] >= (1ull << 62)) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  if (n_entries) *n_entries = 0;
  if (!n) return EWAL_OK;
  EW_CHECK(c->moff.ensure((size_t)n * 8));
  EW_CHECK(c->mlen.ensure((size_t)n * 8));
  EW_CHECK(c->mcnt.ensure((size_t)n * 8));
  EW_CHECK(c->mfirst.ensure((size_t)n * 8));
  EW_CHECK(c->mscnt.ensure((size_t)n * 8));
  EW_CHECK(c->msfirst.ensure((size_t)n * 8));
  EW_CHECK(c->mout.ensure((size_t)n * sizeof(emsg_message)));
  EW_CHECK(hipMemcpyAsync(c->moff.p, offs, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipMemcpyAsync(c->mlen.p, lens, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
  EW_CHECK(hipEventRecord(c->ev0, c->stream));
  const uint8_t *b = (const uint8_t *)d_buf;
  unsigned long long *cnt = c->mcnt.as<unsigned long long>(), *first = c->mfirst.as<unsigned long long>();
  unsigned long long *scnt = c->mscnt.as<unsigned long long>(), *sfirst = c->msfirst.as<unsigned long long>();
  hipLaunchKernelGGL(k_msg<false>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, b, c->moff.as<uint64_t>(),
                     c->mlen.as<uint64_t>(), n, cnt, (const unsigned long long *)nullptr, scnt,
                     (const unsigned long long *)nullptr, (emsg_message *)nullptr, (ewal_entry *)nullptr,
                     (emsg_segment *)nullptr);
  size_t bytes = 0;
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, cnt, first, (int)n, c->stream));
  EW_CHECK(c->tmp.ensure(bytes));
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, bytes, cnt, first, (int)n, c->stream));
  EW_CHECK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, bytes, scnt, sfirst, (int)n, c->stream));
  unsigned long long tail[4];
  EW_CHECK(hipMemcpyAsync(&tail[0], first + (n - 1), 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[1], cnt + (n - 1), 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[2], sfirst + (n - 1), 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipMemcpyAsync(&tail[3], scnt + (n - 1), 8, hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  const uint64_t total = tail[0] + tail[1], stotal = tail[2] + tail[3];
  EW_CHECK(c->ments.ensure((size_t)std::max<uint64_t>(total, 1) * sizeof(ewal_entry)));
  EW_CHECK(c->msegs.ensure((size_t)std::max<uint64_t>(stotal, 1) * sizeof(emsg_segment)));
  hipLaunchKernelGGL(k_msg<true>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, b, c->moff.as<uint64_t>(),
                     c->mlen.as<uint64_t>(), n, cnt, (const unsigned long long *)first, scnt,
                     (const unsigned long long *)sfirst, c->mout.as<emsg_message>(), c->ments.as<ewal_entry>(),
                     c->msegs.as<emsg_segment>());
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipEventRecord(c->ev1, c->stream));
  EW_CHECK(hipMemcpyAsync(out, c->mout.p, (size_t)n * sizeof(emsg_message), hipMemcpyDeviceToHost, c->stream));
  EW_CHECK(hipStreamSynchronize(c->stream));
  c->mtotal = total;
  c->mstotal = stotal;
  if (n_entries) *n_entries = total;
  return EWAL_OK;
}

int64_t emsg_copy_segments(ewal_ctx *c, uint64_t first, emsg_segment *out, int64_t cap) {
  if (!c || (!out && cap) || first > c->mstotal) return EWAL_E_INVAL;
  const int64_t n = std::min<int64_t>(cap, (int64_t)(c->mstotal - first));
  if (n > 0) {
    EW_CHECK(hipMemcpyAsync(out, c->msegs.as<emsg_segment>() + first, (size_t)n * sizeof(emsg_segment),
                            hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
  }
  return n;
}

int64_t emsg_copy_entries(ewal_ctx *c, uint64_t first, ewal_entry *out, int64_t cap) {
  if (!c || (!out && cap) || first > c->mtotal) return EWAL_E_INVAL;
  const int64_t n = std::min<int64_t>(cap, (int64_t)(c->mtotal - first));
  if (n > 0) {
    EW_CHECK(hipMemcpyAsync(out, c->ments.as<ewal_entry>() + first, (size_t)n * sizeof(ewal_entry),
                            hipMemcpyDeviceToHost, c->stream));
    EW_CHECK(hipStreamSynchronize(c->stream));
  }
  return n;
}

float ewal_last_device_ms(ewal_ctx *c) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.f;
  return ms;
}

float ewal_last_stream_ms(ewal_ctx *c) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->evs0, c->evs1) != hipSuccess) return -1.f;
  return ms;
}

int ecommit_batch_device(ewal_ctx *c, uint64_t G, const uint64_t *match, const uint8_t *nvoters, const uint64_t *term,
                         uint64_t *committed, const uint64_t *log_offset, const uint64_t *log_ptr,
                         const uint64_t *log_terms, uint8_t *changed, uint8_t *status, double *device_ms) {
  if (!c) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  EW_CHECK(hipEventRecord(c->ev0, c->stream));
  if (G)
    hipLaunchKernelGGL(k_commit, dim3((unsigned)((G + 256 * EW_COMMIT_ILP - 1) / (256 * EW_COMMIT_ILP))), dim3(256), 0,
                       c->stream, G, match, nvoters, term,
                       committed, log_offset, log_ptr, log_terms, changed, status);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipEventRecord(c->ev1, c->stream));
  EW_CHECK(hipEventSynchronize(c->ev1));
  if (device_ms) {
    float ms = 0;
    EW_CHECK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *device_ms = ms;
  }
  return EWAL_OK;
}

static_assert(sizeof(ecommit_group) == 192, "a group record is 12 16-B loads");
int ecommit_batch_rec_device(ewal_ctx *c, uint64_t G, const ecommit_group *groups, const uint64_t *log_ptr,
                             const uint64_t *log_terms, uint64_t *committed_out, uint8_t *changed, uint8_t *status,
                             double *device_ms) {
  if (!c || (G && (!groups || !committed_out || !changed || !status))) return EWAL_E_INVAL;
  if (((uintptr_t)groups & 15) != 0) return EWAL_E_INVAL;
  EW_CHECK(hipSetDevice(c->device));
  EW_CHECK(hipEventRecord(c->ev0, c->stream));
  if (G)
    hipLaunchKernelGGL(k_commit_rec, dim3((unsigned)std::min<uint64_t>((G + 63) / 64, (uint64_t)std::max(1, c->num_cu) * 12)),
                       dim3(64), 0, c->stream, G, groups, log_ptr,
                       log_terms, committed_out, changed, status);
  EW_CHECK(hipGetLastError());
  EW_CHECK(hipEventRecord(c->ev1, c->stream));
  EW_CHECK(hipEventSynchronize(c->ev1));
  if (device_ms) {
    float ms = 0;
    EW_CHECK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *device_ms = ms;
  }
  return EWAL_OK;
}

}  // extern "C"

#ifdef FR_TIMING
// tools/ timing builds only: the last k_frames launch's per-wave phase cycles
extern "C" int ewal_dbg_fr_timing(unsigned long long *out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fr_tdbg), (size_t)n * 8) != hipSuccess) return EWAL_E_HIP;
  return 0;
}
extern "C" int ewal_dbg_fr_seam_timing(unsigned long long *out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fr_sdbg), (size_t)n * 8) != hipSuccess) return EWAL_E_HIP;
  return 0;
}
extern "C" int ewal_dbg_fr_seam_maxsteps(unsigned long long *out, int n) {   // and zeroes them
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fr_sdbg3), (size_t)n * 8) != hipSuccess) return EWAL_E_HIP;
  std::vector<unsigned long long> z((size_t)n, 0ull);
  if (hipMemcpyToSymbol(HIP_SYMBOL(fr_sdbg3), z.data(), (size_t)n * 8) != hipSuccess) return EWAL_E_HIP;
  return 0;
}
extern "C" int ewal_dbg_fr_result_steps(unsigned long long *out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fr_rdbg), (size_t)std::min(n, 8) * 8) != hipSuccess) return EWAL_E_HIP;
  return 0;
}
extern "C" int ewal_dbg_fr_seam_steps(unsigned long long *out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fr_sdbg2), (size_t)n * 8) != hipSuccess) return EWAL_E_HIP;
  return 0;
}
extern "C" int ewal_dbg_fr_wave_times(unsigned long long *out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fr_wt), (size_t)n * 8) != hipSuccess) return EWAL_E_HIP;
  return 0;
}
#endif
