// msg_kernels.hip -- batched raftpb.Message decode for the /raft ingress
// (SURVEY §8(f) rank 4): raftpb.Message.Unmarshal, raft/raftpb/raft.pb.go:407-617,
// called per POST in etcdserver/etcdhttp/http.go:119-146.  One lane per
// message, two launches: k_msg<false> counts each message's entries and
// segments (so the host can place them with two exclusive scans),
// k_msg<true> decodes every field and writes the entries and segments.  The
// Go semantics kept:
//   * fields 1-6, 8: uint64 varints OR-accumulated (shifts >= 64 give 0);
//   * field 7: Entries = append(Entries, Entry{}); the Entry's Unmarshal
//     error is DISCARDED (raft.pb.go:535 does not check it) but a panic
//     inside it propagates; the partially decoded Entry stays;
//   * field 9: Snapshot.Unmarshal into the same struct (repeats accumulate),
//     its error returns;
//   * field 10: Reject = (v != 0), assigned;
//   * unknown fields: proto.Skip into XXX_unrecognized.
// The byte values Go assembles by append -- every XXX_unrecognized (the
// Message's, each Entry's, the Snapshot's) and a bytes field repeated with
// several non-empty segments (Entry.Data, Snapshot.Data) -- come back as
// segment lists (emsg_segment: ranges of the input whose concatenation is
// the value), and the Snapshot's Nodes / RemovedNodes as value lists.
// EWAL_UNSUPPORTED_ENCODING (48) remains only for protobuf groups nested
// deeper than the device walker's stack.
#include "ewal_device.h"
#include "ewal_internal.h"

// raftpb.Entry / raftpb.Snapshot field sets (bit = field number) for pb_each
#define EMSG_ENTRY_VAR 0x0eu      // Type, Term, Index
#define EMSG_ENTRY_BYTES 0x10u    // Data
#define EMSG_SNAP_VAR 0x3cu       // Nodes, Index, Term, RemovedNodes
#define EMSG_SNAP_BYTES 0x02u     // Data

template <bool FILL>
__device__ int msg_walk(const uint8_t *p, int64_t l, uint64_t base, emsg_message &m, ewal_entry *ents, uint64_t &ne,
                        int &unsup, emsg_segment *segs, uint64_t &ns) {
  auto emit = [&](int32_t kind, int64_t ent, uint64_t off, uint64_t len) {
    if (FILL) {
      emsg_segment g;
      g.kind = kind;
      g.pad = 0;
      g.ent = ent;
      g.off = off;
      g.len = len;
      segs[ns] = g;
    }
    ++ns;
  };
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
      const uint64_t at = base + (uint64_t)i;   // the embedded message's first byte in the buffer
      if (fn == 7) {
        PbField a1, a2, a3, a4, a5;
        pbf_init(a1); pbf_init(a2); pbf_init(a3); pbf_init(a4); pbf_init(a5);
        const int64_t ei = (int64_t)ne;
        const int es = pb_walk<PB_VAR32, PB_VAR64, PB_VAR64, PB_BYTES, PB_NONE>(
            p + i, post - i, a1, a2, a3, a4, a5, unrec, nullptr, nullptr, 0,
            [&](int64_t u0, int64_t u1) { emit(EMSG_SEG_ENTRY_UNREC, ei, at + (uint64_t)u0, (uint64_t)(u1 - u0)); });
        if (es == 33 || es == 37) { st = es; break; }   // panics propagate, errors do not
        if (es == 48) unsup = 1;
        if (a4.split)   // Data = the concatenation of its segments
          pb_each(p + i, post - i, 4, EMSG_ENTRY_VAR, EMSG_ENTRY_BYTES, [&](bool b, uint64_t o, uint64_t n) {
            if (b) emit(EMSG_SEG_ENTRY_DATA, ei, at + o, n);
          });
        if (FILL) {
          ewal_entry e;
          e.type = (int32_t)(uint32_t)a1.v;
          e.term = a2.v;
          e.index = a3.v;
          e.data_nil = a4.split ? 2 : (a4.blen > 0 ? 0 : 1);
          e.data_off = a4.blen > 0 ? at + (uint64_t)a4.boff : 0;
          e.data_len = a4.blen > 0 ? (uint64_t)a4.blen : 0;
          ents[ne] = e;
        }
        ++ne;
      } else {
        const int64_t had = s1.blen;
        const int ss = pb_walk<PB_BYTES, PB_REP64, PB_VAR64, PB_VAR64, PB_REP64>(
            p + i, post - i, s1, s2, s3, s4, s5, unrec, nullptr, nullptr, 0xffffffffu,
            [&](int64_t u0, int64_t u1) { emit(EMSG_SEG_SNAP_UNREC, -1, at + (uint64_t)u0, (uint64_t)(u1 - u0)); });
        if (had == 0 && s1.blen > 0) m.snap_data_off = (int64_t)(at + (uint64_t)s1.boff);
        if (ss == 48) unsup = 1;
        // Nodes, RemovedNodes and the Data segments of this occurrence (they accumulate over repeats)
        if (s2.v) pb_each(p + i, post - i, 2, EMSG_SNAP_VAR, EMSG_SNAP_BYTES, [&](bool b, uint64_t v, uint64_t) {
          if (!b) emit(EMSG_SEG_SNAP_NODE, -1, v, 0);
        });
        if (s5.v) pb_each(p + i, post - i, 5, EMSG_SNAP_VAR, EMSG_SNAP_BYTES, [&](bool b, uint64_t v, uint64_t) {
          if (!b) emit(EMSG_SEG_SNAP_REMOVED, -1, v, 0);
        });
        if (s1.blen > had) pb_each(p + i, post - i, 1, EMSG_SNAP_VAR, EMSG_SNAP_BYTES, [&](bool b, uint64_t o, uint64_t n) {
          if (b) emit(EMSG_SEG_SNAP_DATA, -1, at + o, n);
        });
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
    emit(EMSG_SEG_UNREC, -1, base + (uint64_t)i, (uint64_t)skippy);
    i = hi;
  }
  m.snap_index = s3.v;
  m.snap_term = s4.v;
  m.snap_data_len = s1.blen > 0 ? s1.blen : 0;
  if (s1.split) m.snap_data_off = -2;   // the concatenation of the EMSG_SEG_SNAP_DATA segments
  m.snap_n_nodes = s2.v;
  m.snap_n_removed = s5.v;
  return st;
}

// FILL = false: cnt[k] = entries of message k.  FILL = true: the decoded
// messages, entries at ents[first[k] ..].
template <bool FILL>
__global__ __launch_bounds__(256) void k_msg(const uint8_t *__restrict__ buf, const uint64_t *__restrict__ offs,
                                             const uint64_t *__restrict__ lens, uint32_t n,
                                             unsigned long long *__restrict__ cnt,
                                             const unsigned long long *__restrict__ first,
                                             unsigned long long *__restrict__ scnt,
                                             const unsigned long long *__restrict__ sfirst,
                                             emsg_message *__restrict__ out, ewal_entry *__restrict__ ents,
                                             emsg_segment *__restrict__ segs) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  emsg_message m;
  memset(&m, 0, sizeof(m));
  uint64_t ne = 0, ns = 0;
  int unsup = 0;
  const uint64_t o = offs[k];
  const int st = msg_walk<FILL>(buf + o, (int64_t)lens[k], o, m, FILL ? ents + first[k] : nullptr, ne, unsup,
                                FILL ? segs + sfirst[k] : nullptr, ns);
  if (!FILL) {
    cnt[k] = ne;
    scnt[k] = ns;
    return;
  }
  m.status = st ? st : (unsup ? EWAL_UNSUPPORTED_ENCODING : 0);
  m.ents_first = first[k];
  m.n_ents = ne;
  m.segs_first = sfirst[k];
  m.n_segs = ns;
  out[k] = m;
}
