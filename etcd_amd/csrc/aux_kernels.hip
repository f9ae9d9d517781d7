// aux_kernels.hip -- snapshot CRC batch verify and batched raft quorum commit.
//
//   k_snap    snap.loadSnap (snap/snapshotter.go:76-111): snappb.Snapshot
//             Unmarshal (snap/snappb/snap.pb.go:42-120), crc32.Update(0, tab,
//             Data) against the stored Crc, then raftpb.Snapshot Unmarshal
//             (raft/raftpb/raft.pb.go:279-406).  The CRC of each file's Data
//             comes from the same stream prefixes as the WAL path (k_stream
//             with find_cand = 0 over the packed batch).
//   k_commit  raft.maybeCommit (raft/raft.go:248-258, q() :275-277) +
//             raftLog.maybeCommit / term / at / isOutOfBounds
//             (raft/log.go:115-154, 194-217), one lane per raft group.
#include "ewal_device.h"
#include "ewal_internal.h"

__global__ __launch_bounds__(256) void k_snap(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pwave,
                       const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                       const uint32_t *__restrict__ g_shift, SnapDesc *__restrict__ sd,
                       esnap_snapshot *__restrict__ snaps, uint32_t n) {
  __shared__ uint32_t s_t4[1024];
  __shared__ uint32_t s_svp[1024];   // S_256 (prefix_at's Horner step)
  stage_lds<256>(s_t4, 1024, [&](int i) { return g_slice[i]; });
  stage_lds<256>(s_svp, 1024, [&](int i) { return g_shift[EW_VLOG * 1024 + i]; });
  __syncthreads();
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  SnapDesc d = sd[f];
  PbField a1, a2, a3, a4, a5;
  pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
  int unrec;
  int st = pb_walk<PB_VAR32, PB_BYTES, PB_NONE, PB_NONE, PB_NONE>(buf + d.off, (int64_t)d.len, a1, a2, a3, a4, a5,
                                                                  unrec, nullptr, nullptr, 0);
  d.stored = (uint32_t)a1.v;
  d.doff = d.off + (a2.blen > 0 ? (uint64_t)a2.boff : 0);
  d.dlen = a2.blen > 0 ? (uint64_t)a2.blen : 0;
  d.computed = 0;
  if (st == 0) {
    // crc32.Update(0, crcTable, Data) = S_n(~0 ^ P(s)) ^ P(e) ^ ~0
    if (a2.split) {   // Data = the concatenation of its segments (snap.pb.go append)
      const uint32_t lin = bytes_field_lin(buf + d.off, (int64_t)d.len, 2, d.off, buf, pwave, v, s_t4, s_svp, g_shift);
      d.computed = gshift_n(g_shift, d.dlen, 0xffffffffu) ^ lin ^ 0xffffffffu;
    } else if (d.dlen == 0) {
      d.computed = 0;
    } else {
      const uint32_t Ps = prefix_at(d.doff, pwave, v, buf, s_t4, s_svp);
      const uint32_t Pe = prefix_at(d.doff + d.dlen, pwave, v, buf, s_t4, s_svp);
      d.computed = gshift_n(g_shift, d.dlen, 0xffffffffu ^ Ps) ^ Pe ^ 0xffffffffu;
    }
    if (d.computed != d.stored) {
      st = EWAL_ERR_SNAP_CRC;
    } else if (a2.split) {
      d.resid = 2;   // raftpb.Snapshot over the concatenation: gathered, then k_snap_resid
    } else {
      PbField s1, s2, s3, s4, s5;
      pbf_init(s1); pbf_init(s2); pbf_init(s3); pbf_init(s4); pbf_init(s5);
      esnap_snapshot *o = snaps + f;
      int ur = 0;
      int st2 = d.dlen ? pb_walk<PB_BYTES, PB_REP64, PB_VAR64, PB_VAR64, PB_REP64>(
                             buf + d.doff, (int64_t)d.dlen, s1, s2, s3, s4, s5, ur, o->nodes, o->removed, 64)
                       : 0;
      // Snapshot.XXX_unrecognized, Data in several segments, more Nodes or
      // RemovedNodes than esnap_snapshot holds: k_snap_resid lists them
      if (st2 == 0 && (ur || s1.split || s2.split || s5.split)) d.resid = 1;
      st = st2;
      o->index = s3.v;
      o->term = s4.v;
      o->data_off = s1.blen > 0 ? d.doff + (uint64_t)s1.boff : d.doff;
      o->data_len = s1.blen > 0 ? (uint64_t)s1.blen : 0;
      o->n_nodes = (int64_t)s2.v;
      o->n_removed = (int64_t)s5.v;
    }
  }
  d.st = st;
  sd[f] = d;
}

// ---- residual snapshot encodings (rare; include/ewal.h esnap_copy_field)
// k_snap_gather: one block per listed file whose envelope Data came in
// several segments: the concatenation Go's append builds, into scratch.
__global__ __launch_bounds__(256) void k_snap_gather(const uint8_t *__restrict__ buf, const SnapDesc *__restrict__ sd,
                                                     const uint32_t *__restrict__ rlist,
                                                     const uint64_t *__restrict__ goff, uint8_t *__restrict__ scratch,
                                                     uint32_t nr) {
  const uint32_t r = blockIdx.x;
  if (r >= nr) return;
  const SnapDesc d = sd[rlist[r]];
  if (d.resid != 2) return;
  uint8_t *dst = scratch + goff[r];
  uint64_t pos = 0;
  // snappb.Snapshot: Crc (1) varint, Data (2) bytes
  pb_each(buf + d.off, (int64_t)d.len, 2, 0x2u, 0x4u, [&](bool b, uint64_t o, uint64_t n) {
    if (!b) return;
    const uint8_t *src = buf + d.off + o;
    for (uint64_t j = threadIdx.x; j < n; j += blockDim.x) dst[pos + j] = src[j];
    pos += n;
  });
}

// k_snap_resid: one lane per listed file, raftpb.Snapshot Unmarshal over
// the file's Data (or its gathered concatenation): the FILL pass writes the
// status, esnap_snapshot's fields and the file's segments (emsg_segment:
// offsets into d_buf, or into scratch for a gathered file); the count pass
// only counts the segments.
template <bool FILL>
__global__ __launch_bounds__(256) void k_snap_resid(const uint8_t *__restrict__ buf, const uint8_t *__restrict__ scratch,
                                                    SnapDesc *__restrict__ sd, const uint32_t *__restrict__ rlist,
                                                    const uint64_t *__restrict__ goff, uint32_t nr,
                                                    uint64_t *__restrict__ cnt, const uint64_t *__restrict__ first,
                                                    emsg_segment *__restrict__ segs,
                                                    esnap_snapshot *__restrict__ snaps) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  const uint32_t f = rlist[r];
  SnapDesc d = sd[f];
  const bool gathered = d.resid == 2;
  const uint64_t base = gathered ? goff[r] : d.doff;
  const uint8_t *p = (gathered ? scratch : buf) + base;
  const int64_t l = (int64_t)d.dlen;
  uint64_t ns = 0;
  auto emit = [&](int32_t kind, uint64_t off, uint64_t len) {
    if (FILL) {
      emsg_segment g;
      g.kind = kind;
      g.pad = gathered ? 1 : 0;
      g.ent = -1;
      g.off = off;
      g.len = len;
      segs[first[r] + ns] = g;
    }
    ++ns;
  };
  PbField s1, s2, s3, s4, s5;
  pbf_init(s1); pbf_init(s2); pbf_init(s3); pbf_init(s4); pbf_init(s5);
  esnap_snapshot *o = snaps + f;
  int ur = 0;
  const int st = pb_walk<PB_BYTES, PB_REP64, PB_VAR64, PB_VAR64, PB_REP64>(
      p, l, s1, s2, s3, s4, s5, ur, FILL ? o->nodes : nullptr, FILL ? o->removed : nullptr, 64,
      [&](int64_t u0, int64_t u1) { emit(EMSG_SEG_SNAP_UNREC, base + (uint64_t)u0, (uint64_t)(u1 - u0)); });
  pb_each(p, l, 1, 0x3cu, 0x2u, [&](bool b, uint64_t o2, uint64_t n) {
    if (b) emit(EMSG_SEG_SNAP_DATA, base + o2, n);
  });
  if (s2.split) pb_each(p, l, 2, 0x3cu, 0x2u, [&](bool b, uint64_t v, uint64_t) {
    if (!b) emit(EMSG_SEG_SNAP_NODE, v, 0);
  });
  if (s5.split) pb_each(p, l, 5, 0x3cu, 0x2u, [&](bool b, uint64_t v, uint64_t) {
    if (!b) emit(EMSG_SEG_SNAP_REMOVED, v, 0);
  });
  if (!FILL) {
    cnt[r] = ns;
    return;
  }
  o->index = s3.v;
  o->term = s4.v;
  // one contiguous range of the file, else ~0: esnap_copy_field assembles it
  o->data_off = (gathered || s1.split) ? ~0ull : (s1.blen > 0 ? d.doff + (uint64_t)s1.boff : d.doff);
  o->data_len = s1.blen > 0 ? (uint64_t)s1.blen : 0;
  o->n_nodes = (int64_t)s2.v;
  o->n_removed = (int64_t)s5.v;
  d.st = st;
  sd[f] = d;
}

// q-th largest of n <= 16 voters by rank counting (ties handled as Go's sort
// would place them: the value at sorted-descending position q-1).
// q-th largest of the n <= N match indexes of group g (any correct sort of
// raft.go:252's mis gives the same order statistic): rank-select over N
// register slots, so a wave of 5/7-voter groups compares 8 x 8, not 16 x 16.
template <int N>
__device__ __forceinline__ uint64_t quorum_select(const uint64_t *__restrict__ match, uint64_t G, uint64_t g, int n) {
  uint64_t m[N];
#pragma unroll
  for (int v = 0; v < N; ++v) m[v] = v < n ? match[(uint64_t)v * G + g] : 0ull;
  const int q = n / 2 + 1;
  uint64_t mci = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int gt = 0, ge = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      gt += (j < n && m[j] > m[i]);
      ge += (j < n && m[j] >= m[i]);
    }
    if (i < n && gt < q && q <= ge) mci = m[i];
  }
  return mci;
}

// Any voter count (nvoters is a uint8): rank-select straight from memory
// (more than 16 voters is rare; the register forms above cover 5 / 7).
__device__ __noinline__ uint64_t quorum_select_any(const uint64_t *__restrict__ match, uint64_t G, uint64_t g, int n) {
  const int q = n / 2 + 1;
  for (int i = 0; i < n; ++i) {
    const uint64_t mi = match[(uint64_t)i * G + g];
    int gt = 0, ge = 0;
    for (int j = 0; j < n; ++j) {
      const uint64_t mj = match[(uint64_t)j * G + g];
      gt += mj > mi;
      ge += mj >= mi;
    }
    if (gt < q && q <= ge) return mi;
  }
  return 0;
}

// One lane per raft group, EW_COMMIT_ILP groups per lane (g, g + T, ...): the
// loads that do not depend on the voter count (committed, term, the log
// window bounds) are issued for every group of the lane before the first
// match load, so a wave keeps 4x the independent requests in flight (the
// kernel is a chain nvoters -> match -> select -> term gather -> store).
#ifndef EW_COMMIT_ILP
#define EW_COMMIT_ILP 4
#endif
__global__ __launch_bounds__(256) void k_commit(uint64_t G, const uint64_t *__restrict__ match,
                                                const uint8_t *__restrict__ nvoters, const uint64_t *__restrict__ term,
                                                uint64_t *__restrict__ committed,
                                                const uint64_t *__restrict__ log_offset,
                                                const uint64_t *__restrict__ log_ptr,
                                                const uint64_t *__restrict__ log_terms, uint8_t *__restrict__ changed,
                                                uint8_t *__restrict__ status) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int n[EW_COMMIT_ILP];
  uint64_t c[EW_COMMIT_ILP], tm[EW_COMMIT_ILP], off[EW_COMMIT_ILP], p0[EW_COMMIT_ILP], p1[EW_COMMIT_ILP];
#pragma unroll
  for (int k = 0; k < EW_COMMIT_ILP; ++k) {
    const uint64_t g = g0 + (uint64_t)k * T;
    const bool in = g < G;
    n[k] = in ? nvoters[g] : 0;
    c[k] = in ? committed[g] : 0;
    tm[k] = in ? term[g] : 0;
    off[k] = in ? log_offset[g] : 0;
    p0[k] = in ? log_ptr[g] : 0;
    p1[k] = in ? log_ptr[g + 1] : 0;
  }
#pragma unroll
  for (int k = 0; k < EW_COMMIT_ILP; ++k) {
    const uint64_t g = g0 + (uint64_t)k * T;
    if (g >= G) break;
    const int nv = n[k];
    uint8_t chg = 0, st = 0;
    if (nv <= 0) {
      st = EWAL_PANIC_BOUNDS;   // mis[q-1] on an empty slice (raft/raft.go:255)
    } else {
      const uint64_t mci = nv <= 8 ? quorum_select<8>(match, G, g, nv)
                           : nv <= 16 ? quorum_select<16>(match, G, g, nv) : quorum_select_any(match, G, g, nv);
      if (mci > c[k]) {   // raftLog.maybeCommit: term(mci) == Term (raft/log.go:148-154)
        const uint64_t nlog = p1[k] - p0[k];
        const uint64_t last = nlog - 1 + off[k];    // lastIndex(), uint64 wrap
        uint64_t t = 0;
        bool panic = false;
        if (!(mci < off[k] || mci > last)) {        // raftLog.at / isOutOfBounds (raft/log.go:194-217)
          const uint64_t kk = mci - off[k];
          if (kk >= nlog) panic = true; else t = log_terms[p0[k] + kk];
        }
        if (panic) {
          st = EWAL_PANIC_BOUNDS;
        } else if (t == tm[k]) {
          committed[g] = mci;
          chg = 1;
        }
      }
    }
    changed[g] = chg;
    status[g] = st;
  }
}

// The same over one 192-B record per group (ecommit_group: up to 7 voters'
// Match, committed, Term, the log bounds and the terms of the log's last 13
// entries), read with coalesced loads, instead of 7 strided match words and
// a term gather that fetches a whole 128-B line for 8 bytes.  The quorum
// index's term comes from the record's tail window when it is one of the
// last 13 entries (the usual case: the uncommitted tail of a raft log is a
// few appends deep), else from the log_terms gather as in k_commit.
__global__ __launch_bounds__(64) void k_commit_rec(uint64_t G, const ecommit_group *__restrict__ rec,
                                                   const uint64_t *__restrict__ log_ptr,
                                                   const uint64_t *__restrict__ log_terms,
                                                   uint64_t *__restrict__ committed_out,
                                                   uint8_t *__restrict__ changed, uint8_t *__restrict__ status) {
  // one wave per workgroup, persistent over chunks of 64 records (12 KiB):
  // a chunk is read with fully coalesced 16-B loads (a lane reading its own
  // 192-B record directly would touch 64 lines per load instruction) while
  // the previous one is selected from LDS
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  __shared__ v4u s_rec[64 * 12];
  const uint32_t lane = threadIdx.x;
  const uint64_t nchunk = (G + 63) / 64;
  auto load = [&](uint64_t ch, v4u (&x)[12]) {
    const uint64_t g0 = ch * 64;
    const uint64_t n12 = (G - g0 < 64 ? G - g0 : 64) * 12;
    const v4u *src = (const v4u *)(rec + g0);
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const uint32_t i = (uint32_t)k * 64 + lane;
      x[k] = (ch < nchunk && i < n12) ? __builtin_nontemporal_load(src + i) : v4u{0, 0, 0, 0};   // read once
    }
  };
  v4u cur[12], nxt[12];
  uint64_t ch = blockIdx.x;
  load(ch, cur);
  for (; ch < nchunk; ch += gridDim.x) {
    load(ch + gridDim.x, nxt);
#pragma unroll
    for (int k = 0; k < 12; ++k) s_rec[k * 64 + lane] = cur[k];
    __syncthreads();
    const uint64_t g = ch * 64 + lane;
    if (g < G) {
      const uint64_t *w = (const uint64_t *)(s_rec + lane * 12);   // the record's 8-byte words
      const uint64_t c = w[7], tm = w[8], off = w[9], w10 = w[10];
      const uint64_t nlog = (uint32_t)w10;
      const int nv = (int)((w10 >> 32) & 0xff);
      uint8_t chg = 0, st = 0;
      uint64_t cn = c;
      if (nv <= 0) {
        st = EWAL_PANIC_BOUNDS;   // mis[q-1] on an empty slice (raft/raft.go:255)
      } else if (nv > 7) {
        st = EWAL_UNSUPPORTED_ENCODING;   // more voters than a record holds: ecommit_batch_device
      } else {
        uint64_t m[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) m[v] = v < 7 ? w[v] : 0ull;
        const int qn = nv / 2 + 1;
        uint64_t mci = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {   // rank-select: the qn-th largest (quorum_select's rule)
          int gt = 0, ge = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            gt += (j < nv && m[j] > m[i]);
            ge += (j < nv && m[j] >= m[i]);
          }
          if (i < nv && gt < qn && qn <= ge) mci = m[i];
        }
        if (mci > c) {   // raftLog.maybeCommit: term(mci) == Term (raft/log.go:148-154)
          const uint64_t last = nlog - 1 + off;   // lastIndex(), uint64 wrap
          uint64_t t = 0;
          bool panic = false;
          if (!(mci < off || mci > last)) {       // raftLog.at / isOutOfBounds (raft/log.go:194-217)
            const uint64_t kk = mci - off;
            if (kk >= nlog) {
              panic = true;
            } else if (nlog - 1 - kk < 13) {
              t = w[11 + (nlog - 1 - kk)];
            } else if (log_ptr && log_terms) {
              t = log_terms[log_ptr[g] + kk];
            } else {
              st = EWAL_UNSUPPORTED_ENCODING;    // the term lies before the tail window and no log was given
            }
          }
          if (panic) {
            st = EWAL_PANIC_BOUNDS;
          } else if (!st && t == tm) {
            cn = mci;
            chg = 1;
          }
        }
      }
      committed_out[g] = cn;
      changed[g] = chg;
      status[g] = st;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 12; ++k) cur[k] = nxt[k];
  }
}

// ===========================================================================
// Batched encoder.encode of entries (wal/wal.go:248-263 SaveEntry,
// wal/encoder.go:25-37): frame_i = int64 LE len || walpb.Record{Type: 2, Crc:
// c_i, Data: E_i}, E_i = raftpb.Entry.Marshal() (raft/raftpb/raft.pb.go:
// 921-943), c_i = crc32.Update(c_{i-1}, Castagnoli, E_i).  The CRC chain
// runs over the contiguous "data-only" stream E_0 || E_1 || ... (frame
// headers are not in it), so ONE stream pass gives every c_i:
// c_i = ~P(end of E_i) once the stream's first 4 bytes are XORed with
// ~c_{-1} (a reflected CRC register started at r equals one started at 0 over
// the message whose first 4 bytes are XORed with r).
// ===========================================================================
__device__ __forceinline__ uint32_t sov64(uint64_t x) {
  uint32_t n = 1;
  while (x >= 0x80) { x >>= 7; ++n; }
  return n;
}
__device__ __forceinline__ uint32_t put_varint_dev(uint8_t *o, uint64_t v) {
  uint32_t n = 0;
  while (v >= 0x80) { o[n++] = (uint8_t)(v | 0x80); v >>= 7; }
  o[n++] = (uint8_t)v;
  return n;
}
// Entry header 08 v(type) 10 v(term) 18 v(index) 22 v(len) into h (<= 44 B)
__device__ __forceinline__ uint32_t entry_head(uint8_t *h, const ewal_entry &e) {
  uint32_t o = 0;
  h[o++] = 0x08; o += put_varint_dev(h + o, (uint64_t)(int64_t)e.type);
  h[o++] = 0x10; o += put_varint_dev(h + o, e.term);
  h[o++] = 0x18; o += put_varint_dev(h + o, e.index);
  h[o++] = 0x22; o += put_varint_dev(h + o, e.data_len);
  return o;
}

// Wave-cooperative copy of n bytes src -> dst (any alignment): byte stores for
// the unaligned head and tail of dst, dword stores in between (two aligned
// source dwords and v_alignbyte per output dword).  Source reads stay inside
// [src_base, src_base + src_len).
__device__ __forceinline__ void wave_copy(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint64_t n,
                                          const uint8_t *src_base, uint64_t src_len) {
  const int lane = threadIdx.x & 63;
  const uint64_t head = std::min<uint64_t>(n, (4 - ((uintptr_t)dst & 3)) & 3);
  if ((uint64_t)lane < head) dst[lane] = src[lane];
  const uint64_t m = (n - head) >> 2;                     // whole output dwords
  uint32_t *d32 = (uint32_t *)(dst + head);
  const uint8_t *s = src + head;
  const uintptr_t send = (uintptr_t)(src_base + src_len);
  for (uint64_t k = lane; k < m; k += 64) {
    const uint8_t *p = s + 4 * k;
    const uintptr_t a = (uintptr_t)p & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    uint32_t w;
    if (sh == 0) {
      w = *(const uint32_t *)a;
    } else if (a + 8 <= send) {
      w = __builtin_amdgcn_alignbyte(((const uint32_t *)a)[1], ((const uint32_t *)a)[0], sh);
    } else {
      w = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    }
    d32[k] = w;
  }
  const uint64_t t0 = head + 4 * m;
  if ((uint64_t)lane < n - t0) dst[t0 + lane] = src[t0 + lane];
}

// esz[i] = |E_i|
__global__ void k_enc_sizes(const ewal_entry *__restrict__ ents, uint64_t n, uint64_t data_len,
                            uint64_t *__restrict__ esz, uint32_t *__restrict__ errflag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ewal_entry e = ents[i];
  if (e.data_len > data_len || e.data_off > data_len - e.data_len) atomicOr(errflag, 1u);   // outside d_data
  esz[i] = 4 + sov64((uint64_t)(int64_t)e.type) + sov64(e.term) + sov64(e.index) + sov64(e.data_len) + e.data_len;
}

// E_i at xoff[i] of the data-only stream; one wave per entry (grid-stride)
__global__ __launch_bounds__(256) void k_enc_body(const uint8_t *__restrict__ data, uint64_t data_len,
                                                  const ewal_entry *__restrict__ ents, uint64_t n,
                                                  const uint64_t *__restrict__ xoff, uint8_t *__restrict__ es) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nw) {
    const ewal_entry e = ents[i];
    uint8_t h[48];
    const uint32_t hl = entry_head(h, e);
    uint8_t *o = es + xoff[i];
    if ((uint32_t)lane < hl) {
      uint8_t b = 0;
#pragma unroll
      for (int k = 0; k < 48; ++k) b = (k == lane) ? h[k] : b;
      o[lane] = b;
    }
    if (e.data_len) wave_copy(o + hl, data + e.data_off, e.data_len, data, data_len);
  }
}

// XOR the data-only stream's first 4 bytes with r (and back)
__global__ void k_enc_xor4(uint8_t *es, uint32_t r) {
  if (threadIdx.x < 4) es[threadIdx.x] ^= (uint8_t)(r >> (8 * threadIdx.x));
}

// c_i = ~P(end of E_i); frame size fsz[i] = 8 + |Record|
__global__ __launch_bounds__(256) void k_enc_crc(const uint8_t *__restrict__ es, const uint64_t *__restrict__ xoff,
                                                 const uint64_t *__restrict__ esz, uint64_t n,
                                                 const uint32_t *__restrict__ pwave, const uint32_t *__restrict__ v,
                                                 const uint32_t *__restrict__ g_slice,
                                                 const uint32_t *__restrict__ g_shift, uint32_t *__restrict__ crc,
                                                 uint64_t *__restrict__ fsz) {
  __shared__ uint32_t s_t4[1024];
  __shared__ uint32_t s_svp[1024];
  stage_lds<256>(s_t4, 1024, [&](int i) { return g_slice[i]; });
  stage_lds<256>(s_svp, 1024, [&](int i) { return g_shift[EW_VLOG * 1024 + i]; });
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t L = esz[i];
  const uint32_t c = ~prefix_at(xoff[i] + L, pwave, v, es, s_t4, s_svp);
  crc[i] = c;
  fsz[i] = 8 + 1 + 1 + 1 + sov64(c) + 1 + sov64(L) + L;   // 08 02 10 v(c) 1a v(L) E
}

// frame_i at foff[i]: int64 len, 08 02 10 v(c) 1a v(|E_i|), E_i; one wave per entry
__global__ __launch_bounds__(256) void k_enc_frame(const uint8_t *__restrict__ es, uint64_t es_len,
                                                   const uint64_t *__restrict__ xoff,
                                                   const uint64_t *__restrict__ esz, const uint32_t *__restrict__ crc,
                                                   const uint64_t *__restrict__ foff, uint64_t n,
                                                   uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nw) {
    const uint64_t L = esz[i];
    const uint32_t c = crc[i];
    uint8_t h[32];
    uint32_t o = 8;
    h[o++] = 0x08; h[o++] = 0x02;
    h[o++] = 0x10; o += put_varint_dev(h + o, c);
    h[o++] = 0x1a; o += put_varint_dev(h + o, L);
    const uint64_t rec = (uint64_t)(o - 8) + L;             // the int64 length prefix
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = (uint8_t)(rec >> (8 * k));
    uint8_t *dst = out + foff[i];
    if ((uint32_t)lane < o) {
      uint8_t b = 0;
#pragma unroll
      for (int k = 0; k < 32; ++k) b = (k == lane) ? h[k] : b;
      dst[lane] = b;
    }
    wave_copy(dst + o, es + xoff[i], L, es, es_len);
  }
}

// ===========================================================================
// Batched WAL writes: Save (SaveState + SaveEntry, wal/wal.go:248-279) and Cut
// (wal/wal.go:219-238: a crcType record carrying the running CRC, then the
// metadata record) as ONE chained call.  Every save record contributes one
// contiguous chunk to the data-only stream (Entry / HardState marshal, the
// Cut's metadata bytes; a crcType record adds nothing: Data is nil), so ONE
// stream pass gives every chained CRC as in k_enc_*:
//   crc after the chunk ending at x = ~(P'(x) ^ (x < 4 ? R0 >> 8x : 0)),
// P' over the stream whose first min(4, E) bytes are XORed with R0 = ~prev
// (a reflected register started at R0 over k < 4 bytes equals one started at
// 0 over the XORed bytes, then XORed with R0 >> 8k).
// ===========================================================================
__device__ __forceinline__ uint32_t hardstate_head(uint8_t *h, uint64_t term, uint64_t vote, uint64_t commit) {
  uint32_t o = 0;
  h[o++] = 0x08; o += put_varint_dev(h + o, term);
  h[o++] = 0x10; o += put_varint_dev(h + o, vote);
  h[o++] = 0x18; o += put_varint_dev(h + o, commit);
  return o;
}

// chunk size of save record i (0: no chunk -- an empty HardState writes
// nothing, raft.IsEmptyHardState, wal/wal.go:266-268)
__global__ void k_save_sizes(const ewal_save_rec *__restrict__ recs, uint64_t n, uint64_t data_len,
                             uint64_t *__restrict__ esz, uint32_t *__restrict__ errflag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ewal_save_rec r = recs[i];
  uint64_t z = 0;
  const bool hasd = (r.kind == EWAL_SAVE_ENTRY || r.kind == EWAL_SAVE_CUT) && !(r.kind == EWAL_SAVE_CUT && r.data_nil);
  if (hasd && (r.data_len > data_len || r.data_off > data_len - r.data_len)) atomicOr(errflag, 1u);
  if (r.kind == EWAL_SAVE_ENTRY) {
    z = 4 + sov64((uint64_t)(int64_t)r.etype) + sov64(r.a) + sov64(r.b) + sov64(r.data_len) + r.data_len;
  } else if (r.kind == EWAL_SAVE_STATE) {
    if (r.a | r.b | r.c) z = 3 + sov64(r.a) + sov64(r.b) + sov64(r.c);
  } else if (r.kind == EWAL_SAVE_CUT) {
    z = r.data_nil ? 0 : r.data_len;
  } else {
    atomicOr(errflag, 1u);
  }
  esz[i] = z;
}

// chunk i at xoff[i]; one wave per record (grid-stride)
__global__ __launch_bounds__(256) void k_save_body(const uint8_t *__restrict__ data, uint64_t data_len,
                                                   const ewal_save_rec *__restrict__ recs, uint64_t n,
                                                   const uint64_t *__restrict__ xoff, uint8_t *__restrict__ es) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nw) {
    const ewal_save_rec r = recs[i];
    uint8_t h[48];
    uint32_t hl = 0;
    uint64_t dl = 0;
    if (r.kind == EWAL_SAVE_ENTRY) {
      ewal_entry e;
      e.type = r.etype; e.term = r.a; e.index = r.b; e.data_len = r.data_len;
      hl = entry_head(h, e);
      dl = r.data_len;
    } else if (r.kind == EWAL_SAVE_STATE) {
      if (r.a | r.b | r.c) hl = hardstate_head(h, r.a, r.b, r.c);
    } else if (r.kind == EWAL_SAVE_CUT && !r.data_nil) {
      dl = r.data_len;
    }
    uint8_t *o = es + xoff[i];
    if ((uint32_t)lane < hl) {
      uint8_t b = 0;
#pragma unroll
      for (int k = 0; k < 48; ++k) b = (k == lane) ? h[k] : b;
      o[lane] = b;
    }
    if (dl) wave_copy(o + hl, data + r.data_off, dl, data, data_len);
  }
}

// XOR the stream's first min(4, E) bytes with r (and back)
__global__ void k_save_xor4(uint8_t *es, uint64_t E, uint32_t r) {
  if (threadIdx.x < 4 && threadIdx.x < E) es[threadIdx.x] ^= (uint8_t)(r >> (8 * threadIdx.x));
}

__device__ __forceinline__ uint32_t save_crc_at(uint64_t x, uint32_t R0, uint64_t E, const uint32_t *pwave,
                                                const uint32_t *v, const uint8_t *es, const uint32_t *t4,
                                                const uint32_t *svp) {
  const uint32_t p = (E && x) ? prefix_at(x, pwave, v, es, t4, svp) : 0u;
  return ~(p ^ (x < 4 ? (R0 >> (8 * x)) : 0u));
}

// crc[i] = the running CRC after record i's chunk (its Record.Crc), pcrc[i]
// = before it (a Cut's crcType record); fsz[i] = bytes of record i's frames
__global__ __launch_bounds__(256) void k_save_crc(const uint8_t *__restrict__ es, uint64_t E,
                                                  const ewal_save_rec *__restrict__ recs,
                                                  const uint64_t *__restrict__ xoff, const uint64_t *__restrict__ esz,
                                                  uint64_t n, uint32_t R0, const uint32_t *__restrict__ pwave,
                                                  const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                                                  const uint32_t *__restrict__ g_shift, uint32_t *__restrict__ crc,
                                                  uint32_t *__restrict__ pcrc, uint64_t *__restrict__ fsz) {
  __shared__ uint32_t s_t4[1024];
  __shared__ uint32_t s_svp[1024];
  stage_lds<256>(s_t4, 1024, [&](int i) { return g_slice[i]; });
  stage_lds<256>(s_svp, 1024, [&](int i) { return g_shift[EW_VLOG * 1024 + i]; });
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ewal_save_rec r = recs[i];
  const uint64_t L = esz[i];
  const uint32_t c = save_crc_at(xoff[i] + L, R0, E, pwave, v, es, s_t4, s_svp);
  crc[i] = c;
  uint64_t f = 0;
  if (r.kind == EWAL_SAVE_ENTRY || (r.kind == EWAL_SAVE_STATE && L)) {
    f = 8 + 1 + 1 + 1 + sov64(c) + 1 + sov64(L) + L;              // 08 t 10 v(c) 1a v(L) chunk
  } else if (r.kind == EWAL_SAVE_CUT) {
    const uint32_t c0 = save_crc_at(xoff[i], R0, E, pwave, v, es, s_t4, s_svp);
    pcrc[i] = c0;
    f = 8 + 1 + 1 + 1 + sov64(c0);                                 // crcType: 08 04 10 v(c0), Data nil
    f += 8 + 1 + 1 + 1 + sov64(c) + (r.data_nil ? 0 : 1 + sov64(L) + L);   // metadataType
  }
  fsz[i] = f;
}

// one frame (int64 len || 08 t 10 v(c) [1a v(L) chunk]) at dst; one wave
__device__ __forceinline__ void save_frame(uint8_t *dst, int32_t t, uint32_t c, bool hasd, const uint8_t *chunk,
                                           uint64_t L, const uint8_t *es, uint64_t es_len) {
  const int lane = threadIdx.x & 63;
  uint8_t h[32];
  uint32_t o = 8;
  h[o++] = 0x08; h[o++] = (uint8_t)t;
  h[o++] = 0x10; o += put_varint_dev(h + o, c);
  if (hasd) { h[o++] = 0x1a; o += put_varint_dev(h + o, L); }
  const uint64_t rec = (uint64_t)(o - 8) + (hasd ? L : 0);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = (uint8_t)(rec >> (8 * k));
  if ((uint32_t)lane < o) {
    uint8_t b = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) b = (k == lane) ? h[k] : b;
    dst[lane] = b;
  }
  if (hasd && L) wave_copy(dst + o, chunk, L, es, es_len);
}

__global__ __launch_bounds__(256) void k_save_frame(const uint8_t *__restrict__ es, uint64_t es_len,
                                                    const ewal_save_rec *__restrict__ recs,
                                                    const uint64_t *__restrict__ xoff, const uint64_t *__restrict__ esz,
                                                    const uint32_t *__restrict__ crc, const uint32_t *__restrict__ pcrc,
                                                    const uint64_t *__restrict__ foff, uint64_t n,
                                                    uint8_t *__restrict__ out) {
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nw) {
    const ewal_save_rec r = recs[i];
    const uint64_t L = esz[i];
    uint8_t *dst = out + foff[i];
    if (r.kind == EWAL_SAVE_ENTRY || (r.kind == EWAL_SAVE_STATE && L)) {
      save_frame(dst, r.kind == EWAL_SAVE_ENTRY ? 2 : 3, crc[i], true, es + xoff[i], L, es, es_len);
    } else if (r.kind == EWAL_SAVE_CUT) {
      const uint32_t c0 = pcrc[i];
      save_frame(dst, 4, c0, false, nullptr, 0, es, es_len);
      dst += 8 + 1 + 1 + 1 + sov64(c0);
      save_frame(dst, 1, crc[i], !r.data_nil, es + xoff[i], L, es, es_len);
    }
  }
}
