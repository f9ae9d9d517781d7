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

__constant__ uint8_t c_kind_snappb[8] = {0, PB_VAR32, PB_BYTES, 0, 0, 0, 0, 0};
__constant__ uint8_t c_kind_snapshot[8] = {0, PB_BYTES, PB_REP64, PB_VAR64, PB_VAR64, PB_REP64, 0, 0};

__device__ __forceinline__ uint32_t prefix_at_g(uint64_t x, const uint32_t *__restrict__ pwave,
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

__global__ void k_snap(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pwave,
                       const uint32_t *__restrict__ v, const uint32_t *__restrict__ g_slice,
                       const uint32_t *__restrict__ g_shift, SnapDesc *__restrict__ sd,
                       esnap_snapshot *__restrict__ snaps, uint32_t n) {
  __shared__ uint32_t s_t4[1024];
  __shared__ uint32_t s_s64[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
    s_t4[i] = g_slice[i];
    s_s64[i] = g_shift[6 * 1024 + i];
  }
  __syncthreads();
  uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  SnapDesc d = sd[f];
  PbOut o;
  pb_init(o);
  int st = pb_walk(buf + d.off, (int64_t)d.len, c_kind_snappb, o, nullptr, 0);
  d.stored = (uint32_t)o.v[1];
  d.doff = d.off + (o.blen[2] > 0 ? (uint64_t)o.boff[2] : 0);
  d.dlen = o.blen[2] > 0 ? (uint64_t)o.blen[2] : 0;
  d.computed = 0;
  if (st == 0) {
    // crc32.Update(0, crcTable, Data) = S_n(~0 ^ P(s)) ^ P(e) ^ ~0
    if (d.dlen == 0) {
      d.computed = 0;
    } else {
      const uint32_t Ps = prefix_at_g(d.doff, pwave, v, buf, s_t4, s_s64);
      const uint32_t Pe = prefix_at_g(d.doff + d.dlen, pwave, v, buf, s_t4, s_s64);
      d.computed = gshift_n(g_shift, d.dlen, 0xffffffffu ^ Ps) ^ Pe ^ 0xffffffffu;
    }
    if (d.computed != d.stored) {
      st = EWAL_ERR_SNAP_CRC;
    } else {
      PbOut s;
      pb_init(s);
      uint64_t rep[128];
      int s2 = d.dlen ? pb_walk(buf + d.doff, (int64_t)d.dlen, c_kind_snapshot, s, rep, 64) : 0;
      if (s2 == 0 && s.unrec) s2 = EWAL_UNSUPPORTED_ENCODING;  // Snapshot.XXX_unrecognized is returned
      st = s2;
      esnap_snapshot out;
      out.index = s.v[3];
      out.term = s.v[4];
      out.data_off = s.blen[1] > 0 ? d.doff + (uint64_t)s.boff[1] : d.doff;
      out.data_len = s.blen[1] > 0 ? (uint64_t)s.blen[1] : 0;
      out.n_nodes = s.nrep[2];
      out.n_removed = s.nrep[5];
      for (int k = 0; k < 64; ++k) {
        out.nodes[k] = k < (int)s.nrep[2] ? rep[k] : 0;
        out.removed[k] = k < (int)s.nrep[5] ? rep[64 + k] : 0;
      }
      if (snaps) snaps[f] = out;
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
