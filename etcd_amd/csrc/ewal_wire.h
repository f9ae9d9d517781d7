// ewal_wire.h -- the protobuf MarshalTo forms of etcd's generated code that
// the host writers need (walpb.Record, raftpb.Entry / HardState), shared by
// the engine's writer (ewal_host.cpp) and the synthetic-WAL generator
// (ewal_synth.cpp, bench / test plumbing).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace ewal_wire {

inline size_t sov(uint64_t x) { size_t n = 0; do { n++; x >>= 7; } while (x); return n; }
inline uint8_t *put_varint(uint8_t *o, uint64_t v) {
  while (v >= 0x80) { *o++ = (uint8_t)(v | 0x80); v >>= 7; }
  *o++ = (uint8_t)v;
  return o;
}
// raftpb.Entry.MarshalTo, raft/raftpb/raft.pb.go:921-943
inline size_t entry_size(int32_t type, uint64_t term, uint64_t index, uint64_t n) {
  return 1 + sov((uint64_t)(int64_t)type) + 1 + sov(term) + 1 + sov(index) + 1 + sov(n) + n;
}
inline uint8_t *entry_marshal(uint8_t *o, int32_t type, uint64_t term, uint64_t index, const uint8_t *d, uint64_t n) {
  *o++ = 0x08; o = put_varint(o, (uint64_t)(int64_t)type);
  *o++ = 0x10; o = put_varint(o, term);
  *o++ = 0x18; o = put_varint(o, index);
  *o++ = 0x22; o = put_varint(o, n);
  if (n) std::memcpy(o, d, n);
  return o + n;
}
// raftpb.HardState.MarshalTo, raft.pb.go:1079-1097
inline size_t state_marshal(uint8_t *o, uint64_t term, uint64_t vote, uint64_t commit) {
  uint8_t *s = o;
  *o++ = 0x08; o = put_varint(o, term);
  *o++ = 0x10; o = put_varint(o, vote);
  *o++ = 0x18; o = put_varint(o, commit);
  return (size_t)(o - s);
}
// walpb.Record.MarshalTo, wal/walpb/record.pb.go:175-196, prefixed by the
// int64 LE length (wal/encoder.go:32-35).
inline size_t frame_size(int64_t type, uint32_t crc, uint64_t n, bool nil) {
  size_t r = 1 + sov((uint64_t)type) + 1 + sov(crc);
  if (!nil) r += 1 + sov(n) + n;
  return 8 + r;
}
inline uint8_t *frame_write(uint8_t *o, int64_t type, uint32_t crc, const uint8_t *d, uint64_t n, bool nil) {
  int64_t L = (int64_t)frame_size(type, crc, n, nil) - 8;
  std::memcpy(o, &L, 8);
  o += 8;
  *o++ = 0x08; o = put_varint(o, (uint64_t)type);
  *o++ = 0x10; o = put_varint(o, crc);
  if (!nil) {
    *o++ = 0x1a; o = put_varint(o, n);
    if (n) std::memcpy(o, d, n);
    o += n;
  }
  return o;
}

}  // namespace ewal_wire
