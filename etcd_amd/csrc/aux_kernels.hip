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
    if (d.dlen == 0) {
      d.computed = 0;
    } else {
      const uint32_t Ps = prefix_at(d.doff, pwave, v, buf, s_t4, s_svp);
      const uint32_t Pe = prefix_at(d.doff + d.dlen, pwave, v, buf, s_t4, s_svp);
      d.computed = gshift_n(g_shift, d.dlen, 0xffffffffu ^ Ps) ^ Pe ^ 0xffffffffu;
    }
    if (d.computed != d.stored) {
      st = EWAL_ERR_SNAP_CRC;
    } else {
      PbField s1, s2, s3, s4, s5;
      pbf_init(s1); pbf_init(s2); pbf_init(s3); pbf_init(s4); pbf_init(s5);
      esnap_snapshot *o = snaps + f;
      int ur = 0;
      int st2 = d.dlen ? pb_walk<PB_BYTES, PB_REP64, PB_VAR64, PB_VAR64, PB_REP64>(
                             buf + d.doff, (int64_t)d.dlen, s1, s2, s3, s4, s5, ur, o->nodes, o->removed, 64)
                       : 0;
      if (st2 == 0 && ur) st2 = EWAL_UNSUPPORTED_ENCODING;  // Snapshot.XXX_unrecognized is returned
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

// q-th largest of n <= 16 voters by rank counting (ties handled as Go's sort
// would place them: the value at sorted-descending position q-1).
__global__ void k_commit(uint64_t G, const uint64_t *__restrict__ match, const uint8_t *__restrict__ nvoters,
                         const uint64_t *__restrict__ term, uint64_t *__restrict__ committed,
                         const uint64_t *__restrict__ log_offset, const uint64_t *__restrict__ log_ptr,
                         const uint64_t *__restrict__ log_terms, uint8_t *__restrict__ changed,
                         uint8_t *__restrict__ status) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int n = nvoters[g];
  uint8_t chg = 0, st = 0;
  if (n <= 0 || n > 16) {
    st = EWAL_PANIC_BOUNDS;   // mis[q-1] on an empty slice (n == 0); n > 16 unsupported
  } else {
    uint64_t m[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) m[v] = v < n ? match[(uint64_t)v * G + g] : 0ull;
    const int q = n / 2 + 1;
    uint64_t mci = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int gt = 0, ge = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        gt += (j < n && m[j] > m[i]);
        ge += (j < n && m[j] >= m[i]);
      }
      if (i < n && gt < q && q <= ge) mci = m[i];
    }
    uint64_t c = committed[g];
    if (mci > c) {
      const uint64_t off = log_offset[g];
      const uint64_t p0 = log_ptr[g];
      const uint64_t nlog = log_ptr[g + 1] - p0;
      const uint64_t last = nlog - 1 + off;    // lastIndex(), uint64 wrap
      uint64_t t = 0;
      bool panic = false;
      if (!(mci < off || mci > last)) {
        const uint64_t k = mci - off;
        if (k >= nlog) panic = true; else t = log_terms[p0 + k];
      }
      if (panic) {
        st = EWAL_PANIC_BOUNDS;
      } else if (t == term[g]) {
        committed[g] = mci;
        chg = 1;
      }
    }
  }
  changed[g] = chg;
  status[g] = st;
}
