// ewal_synth.cpp -- the synthetic WAL generator of bench.py and the tests
// (libewal_synth.so, include/ewal_synth.h).  Test and bench plumbing: it is
// not part of the product library (libewal.so) and the engine never calls it.
// It writes what the reference's writer would (wal.Create + Save, the frame
// layout of wal/encoder.go:25-37), with the chained CRC from libewal's
// host pkg/crc helpers (ewal_crc32_update_host / ewal_crc32_combine).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/ewal.h"
#include "../../include/ewal_synth.h"
#include "ewal_wire.h"

using namespace ewal_wire;

namespace {
const uint32_t kCastagnoli = 0x82F63B78u;
}

extern "C" {

// ---- synthetic WAL generator -------------------------------------------------
// Create(Info{ID:1}) + Save(HardState{Term:1,Vote:1}, ents) where ents[i] =
// Entry{Type:0, Term:1, Index:i+1, Data: len_i bytes}, len_i log-uniform in
// [min_data, max_data] and the payload from xorshift64* seeded per entry.
// With rewind_per_mille > 0, that share of the entries open a new leader's
// term that rewrites the last 1..8 indexes (the uncommitted tail a new leader
// overwrites: ReadAll's ents = append(ents[:Index-ri], e), wal/wal.go:173).
// Two parallel passes: (1) CRC-32C of each entry's marshalled bytes,
// (2) layout from the chained CRCs (varint widths), then bytes in place.
static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void fill_payload(uint8_t *o, uint64_t n, uint64_t seed) {
  uint64_t x = mix64(seed) | 1;
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    uint64_t v = x * 0x2545F4914F6CDD1Dull;
    std::memcpy(o + i, &v, 8);
  }
  if (i < n) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    uint64_t v = x * 0x2545F4914F6CDD1Dull;
    std::memcpy(o + i, &v, (size_t)(n - i));
  }
}

int64_t ewal_synth_wal(uint64_t seed, uint64_t target, uint32_t min_data, uint32_t max_data, int64_t corrupt_record,
                       uint8_t *out, uint64_t cap, int64_t *n_records) {
  return ewal_synth_wal_ex(seed, target, min_data, max_data, corrupt_record, 0, out, cap, n_records, nullptr);
}

int64_t ewal_synth_wal_ex(uint64_t seed, uint64_t target, uint32_t min_data, uint32_t max_data,
                          int64_t corrupt_record, uint32_t rewind_per_mille, uint8_t *out, uint64_t cap,
                          int64_t *n_records, uint64_t *last_index) {
  if (min_data == 0 || max_data < min_data || rewind_per_mille > 1000) return EWAL_E_INVAL;
  // entry sizes
  std::vector<uint32_t> sz;
  const double lo = std::log((double)min_data), hi = std::log((double)max_data + 1.0);
  uint64_t rng = mix64(seed ^ 0x5157A11ull);
  uint64_t approx = 64;
  while (approx < target) {
    rng = mix64(rng);
    double u = (double)(rng >> 11) * (1.0 / 9007199254740992.0);
    uint32_t s = (uint32_t)std::exp(lo + u * (hi - lo));
    s = std::min(std::max(s, min_data), max_data);
    sz.push_back(s);
    approx += 8 + 2 + 5 + 1 + sov(s + 32) + entry_size(0, 1, sz.size(), s);
  }
  const size_t N = sz.size();
  // each entry's Term and Index (a new leader's term rewinds the index)
  std::vector<uint64_t> eterm(N), eidx(N);
  {
    uint64_t term = 1, idx = 0, r2 = mix64(seed ^ 0xBEEFull);
    for (size_t j = 0; j < N; ++j) {
      r2 = mix64(r2);
      if (rewind_per_mille && j > 8 && (r2 % 1000) < rewind_per_mille) {
        ++term;
        const uint64_t back = 1 + ((r2 >> 20) & 7);
        idx = idx > back ? idx - back : 0;
      }
      eterm[j] = term;
      eidx[j] = ++idx;
    }
    if (last_index) *last_index = N ? eidx[N - 1] : 0;
  }
  const uint8_t md[2] = {0x08, 0x01};   // etcdserverpb.Info{ID: 1}
  uint8_t st[40];
  const size_t stn = state_marshal(st, 1, 1, 0);
  // pass 1: Update(0, entry bytes) per entry, in parallel
  std::vector<uint32_t> ecrc(N);
  unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  {
    std::atomic<size_t> next(0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nth; ++t)
      th.emplace_back([&]() {
        std::vector<uint8_t> tmp;
        for (;;) {
          size_t i = next.fetch_add(256);
          if (i >= N) break;
          for (size_t j = i; j < std::min(N, i + 256); ++j) {
            tmp.resize(entry_size(0, eterm[j], eidx[j], sz[j]));
            uint8_t *o = tmp.data();
            *o++ = 0x08; o = put_varint(o, 0);
            *o++ = 0x10; o = put_varint(o, eterm[j]);
            *o++ = 0x18; o = put_varint(o, eidx[j]);
            *o++ = 0x22; o = put_varint(o, sz[j]);
            fill_payload(o, sz[j], seed * 1000003ull + j);
            ecrc[j] = ewal_crc32_update_host(0, kCastagnoli, tmp.data(), tmp.size());
          }
        }
      });
    for (auto &x : th) x.join();
  }
  // pass 2 (serial, O(N)): chained CRCs and frame offsets
  std::vector<uint64_t> foff(N);
  std::vector<uint32_t> fcrc(N);
  uint32_t c = 0;
  uint64_t off = 0;
  // crc record, metadata, state
  const uint32_t c_crc = c;
  off += frame_size(4, c_crc, 0, true);
  c = ewal_crc32_update_host(c, kCastagnoli, md, 2);
  const uint32_t c_md = c;
  off += frame_size(1, c_md, 2, false);
  c = ewal_crc32_update_host(c, kCastagnoli, st, stn);
  const uint32_t c_st = c;
  off += frame_size(3, c_st, stn, false);
  const uint64_t head = off;
  for (size_t j = 0; j < N; ++j) {
    const uint64_t en = entry_size(0, eterm[j], eidx[j], sz[j]);
    c = ewal_crc32_combine(kCastagnoli, c, ecrc[j], en);
    fcrc[j] = c;
    foff[j] = off;
    off += frame_size(2, c, en, false);
  }
  if (off > cap) return EWAL_E_NOMEM;
  // write head frames
  uint8_t *o = out;
  o = frame_write(o, 4, c_crc, nullptr, 0, true);
  o = frame_write(o, 1, c_md, md, 2, false);
  o = frame_write(o, 3, c_st, st, stn, false);
  (void)head;
  // pass 3: frames in place, in parallel
  {
    std::atomic<size_t> next(0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nth; ++t)
      th.emplace_back([&]() {
        for (;;) {
          size_t i = next.fetch_add(256);
          if (i >= N) break;
          for (size_t j = i; j < std::min(N, i + 256); ++j) {
            const uint64_t en = entry_size(0, eterm[j], eidx[j], sz[j]);
            uint8_t *f = out + foff[j];
            int64_t L = (int64_t)frame_size(2, fcrc[j], en, false) - 8;
            std::memcpy(f, &L, 8);
            uint8_t *p = f + 8;
            *p++ = 0x08; p = put_varint(p, 2);
            *p++ = 0x10; p = put_varint(p, fcrc[j]);
            *p++ = 0x1a; p = put_varint(p, en);
            *p++ = 0x08; p = put_varint(p, 0);
            *p++ = 0x10; p = put_varint(p, eterm[j]);
            *p++ = 0x18; p = put_varint(p, eidx[j]);
            *p++ = 0x22; p = put_varint(p, sz[j]);
            fill_payload(p, sz[j], seed * 1000003ull + j);
            if ((int64_t)(j + 3) == corrupt_record) p[sz[j] / 2] ^= 0x5a;
          }
        }
      });
    for (auto &x : th) x.join();
  }
  if (n_records) *n_records = (int64_t)(N + 3);
  return (int64_t)off;
}

}  // extern "C"
