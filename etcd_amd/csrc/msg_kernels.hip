// msg_kernels.hip -- batched raftpb.Message decode for the /raft ingress
// (SURVEY §8(f) rank 4): raftpb.Message.Unmarshal, raft/raftpb/raft.pb.go:407-617,
// called per POST in etcdserver/etcdhttp/http.go:119-146.  One lane per
// message, two launches: k_msg<false> counts each message's entries (so
// the host can place them with one exclusive scan), k_msg<true> decodes
// every field and writes the entries.  The Go semantics kept:
//   * fields 1-6, 8: uint64 varints OR-accumulated (shifts >= 64 give 0);
//   * field 7: Entries = append(Entries, Entry{}); the Entry's Unmarshal
//     error is DISCARDED (raft.pb.go:535 does not check it) but a panic
//     inside it propagates; the partially decoded Entry stays;
//   * field 9: Snapshot.Unmarshal into the same struct (repeats accumulate),
//     its error returns;
//   * field 10: Reject = (v != 0), assigned;
//   * unknown fields: proto.Skip into XXX_unrecognized.
// EWAL_UNSUPPORTED_ENCODING (48) -- reported, never guessed -- when the
// decoded value would carry bytes this layout does not return: a Message /
// Entry / Snapshot XXX_unrecognized, or a bytes field repeated with two
// non-empty segments.
#include "ewal_device.h"
#include "ewal_internal.h"

template <bool FILL>
__device__ int msg_walk(const uint8_t *p, int64_t l, uint64_t base, emsg_message &m, ewal_entry *ents, uint64_t &ne,
                        int &unsup) {
  int64_t i = 0;
  PbField s1, s2, s3, s4, s5;   // the Snapshot, accumulated over repeats
  pbf_init(s1); pbf_init(s2); pbf_init(s3); pbf_init(s4); pbf_init(s5);
  m.snap_data_off = -1;
  int st = 0;
  while (i < l) {
    uint64_t wire = 0;
    if (rd_varint(p, i, l, wire, 64)) { st = 2; break; }
    const uint32_t fn = (uint32_t)(wire >> 3);
    const int wt = (int)(wire & 7);
    if ((fn >= 1 && fn <= 6) || fn == 8) {
      if (wt != 0) { st = 7; break; }
      // m.X |= chunk << shift per byte == m.X |= the varint's value, also
      // for the bits read before a truncation (Go leaves them in the field)
      uint64_t v = 0;
      const int e = rd_varint(p, i, l, v, 64);
      switch (fn) {   // named fields, no pointer into m (it stays in registers)
      case 1: m.type |= v; break;
      case 2: m.to |= v; break;
      case 3: m.from |= v; break;
      case 4: m.term |= v; break;
      case 5: m.log_term |= v; break;
      case 6: m.index |= v; break;
      default: m.commit |= v; break;
      }
      if (e) { st = 2; break; }
      continue;
    }
    if (fn == 7 || fn == 9) {
      if (wt != 2) { st = 7; break; }
      uint64_t ml = 0;
      if (rd_varint(p, i, l, ml, 64)) { st = 2; break; }
      const int64_t post = (int64_t)((uint64_t)i + ml);
      if (post > l) { st = 2; break; }
      if (post < i) { st = 33; break; }   // data[index:postIndex]
      int unrec = 0;
      if (fn == 7) {
        PbField a1, a2, a3, a4, a5;
        pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
        const int es = pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(p + i, post - i, a1, a2, a3, a4, a5,
                                                                               unrec, nullptr, nullptr, 0);
        if (es == 33 || es == 37) { st = es; break; }   // panics propagate, errors do not
        if (es == 48 || unrec || a4.split) unsup = 1;
        if (FILL) {
          ewal_entry e;
          e.type = (int32_t)(uint32_t)a1.v;
          e.term = a2.v;
          e.index = a3.v;
          e.data_nil = a4.blen > 0 ? 0 : 1;
          e.data_off = a4.blen > 0 ? base + (uint64_t)i + (uint64_t)a4.boff : 0;
          e.data_len = a4.blen > 0 ? (uint64_t)a4.blen : 0;
          ents[ne] = e;
        }
        ++ne;
      } else {
        const int64_t had = s1.blen;
        const int ss = pb_walk<PB_BYTES, PB_REP64, PB_VAR64, PB_VAR64, PB_REP64>(p + i, post - i, s1, s2, s3, s4, s5,
                                                                                unrec, nullptr, nullptr, 0xffffffffu);
        if (had == 0 && s1.blen > 0) m.snap_data_off = (int64_t)(base + (uint64_t)i + (uint64_t)s1.boff);
        if (unrec || s1.split) unsup = 1;
        if (ss) { st = ss; break; }
      }
      i = post;
      continue;
    }
    if (fn == 10) {
      if (wt != 0) { st = 7; break; }
      uint64_t v = 0;
      if (rd_varint(p, i, l, v, 64)) { st = 2; break; }
      m.reject = v != 0;
      continue;
    }
    // default: index -= sizeOfWire; Skip(data[index:]); XXX_unrecognized
    int64_t sow = 0;
    uint64_t w = wire;
    do { ++sow; w >>= 7; } while (w);
    i -= sow;
    int64_t skippy;
    const int ks = pb_skip(p + i, l - i, skippy);
    if (ks) { st = ks; break; }
    const int64_t hi = (int64_t)((uint64_t)i + (uint64_t)skippy);
    if (hi > l) { st = 2; break; }
    if (hi < i) { st = 33; break; }
    if (skippy == 0) { st = 37; break; }
    m.unrec_len += skippy;
    i = hi;
  }
  m.snap_index = s3.v;
  m.snap_term = s4.v;
  m.snap_data_len = s1.blen > 0 ? s1.blen : 0;
  m.snap_n_nodes = s2.v;
  m.snap_n_removed = s5.v;
  if (m.unrec_len) unsup = 1;
  return st;
}

// FILL = false: cnt[k] = entries of message k.  FILL = true: the decoded
// messages, entries at ents[first[k] ..].
template <bool FILL>
__global__ __launch_bounds__(256) void k_msg(const uint8_t *__restrict__ buf, const uint64_t *__restrict__ offs,
                                             const uint64_t *__restrict__ lens, uint32_t n,
                                             unsigned long long *__restrict__ cnt,
                                             const unsigned long long *__restrict__ first,
                                             emsg_message *__restrict__ out, ewal_entry *__restrict__ ents) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  emsg_message m;
  memset(&m, 0, sizeof(m));
  uint64_t ne = 0;
  int unsup = 0;
  const uint64_t o = offs[k];
  const int st = msg_walk<FILL>(buf + o, (int64_t)lens[k], o, m, FILL ? ents + first[k] : nullptr, ne, unsup);
  if (!FILL) {
    cnt[k] = ne;
    return;
  }
  m.status = st ? st : (unsup ? EWAL_UNSUPPORTED_ENCODING : 0);
  m.ents_first = first[k];
  m.n_ents = ne;
  out[k] = m;
}
