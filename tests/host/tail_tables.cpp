// Host check of the frame pass's shift tables (crc_math.h EW_TAIL_TABS) and
// of the identities its prefix and check code rely on (wal_kernels.hip
// prefix_near_tail / tail_shift, frame_kernels.hip S_dlen), against direct
// CRC-32C register arithmetic.  Exit 0 and "ok" when every case holds.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "crc_math.h"

using ewal::CrcTables;

static uint32_t nib(const uint32_t *t, uint32_t x) {
  uint32_t r = 0;
  for (int k = 0; k < 8; k++) r ^= t[k * 16 + ((x >> (4 * k)) & 15)];
  return r;
}

int main() {
  CrcTables T(0x82f63b78u);
  const uint32_t *tt = &T.shift[EW_TAIL_OFF];
  std::mt19937 g(11);
  long bad = 0;
  // every table is the shift its index names
  for (int t = 0; t < EW_TAIL_TABS; t++)
    for (int i = 0; i < 64; i++) {
      const uint32_t x = g();
      if (nib(tt + t * 128, x) != T.shift_signed(ew_tail_amount(t), x)) bad++;
    }
  // tail_shift: two rounds, forward or back, |s| <= 128
  for (int s = -128; s <= 128; s++)
    for (int i = 0; i < 32; i++) {
      const uint32_t x = g(), u = (uint32_t)(s < 0 ? -s : s);
      const uint32_t *t1 = tt + ((s < 0 ? 34u : 9u) + (u & 15)) * 128, *t2 = tt + ((s < 0 ? 25u : 0u) + (u >> 4)) * 128;
      if (nib(t2, nib(t1, x)) != T.shift_signed(s, x)) bad++;
    }
  // the masked-block tail: P(x) from x0 forward or from x1 = x0 + 256 back
  std::vector<uint8_t> buf(256);
  for (int trial = 0; trial < 20; trial++) {
    for (auto &c : buf) c = (uint8_t)g();
    const uint32_t acc0 = g(), acc1 = T.raw(acc0, buf.data(), 256);
    for (int x = 0; x < 256; x++) {
      const uint32_t P = T.raw(acc0, buf.data(), x);
      uint8_t blk[128] = {0};
      uint32_t r;
      if (x <= 128) {
        std::memcpy(blk, buf.data(), x);
        r = T.shift_signed(x, acc0) ^ T.shift_signed(-(128 - x), T.raw(0, blk, 128));
      } else {
        const int base = x & ~15, lead = x & 15, n = 256 - base;
        std::memcpy(blk + lead, buf.data() + x, 256 - x);
        r = T.shift_signed(-(n - lead), acc1) ^ T.shift_signed(-(128 - lead), T.raw(0, blk, 128));
      }
      if (r != P) bad++;
    }
  }
  // the checks' S_dlen: the low 12 bits in three table rounds, the rest by powers of two
  for (int i = 0; i < 200000; i++) {
    const uint64_t m = g() % (1u << 20);
    const uint32_t x = g(), lo4 = m & 15, a4 = (m >> 4) & 15, h4 = (m >> 8) & 15;
    uint32_t y = nib(tt + (9 + lo4) * 128, x);
    y = nib(tt + (a4 <= 8 ? a4 : 41 + a4) * 128, y);
    y = nib(tt + (h4 ? 56 + h4 : 0) * 128, y);
    y = T.shift_n(m >> 12 << 12, y);
    if (y != T.shift_n(m, x)) bad++;
  }
  // the seam pass's digit tables (seam_shift): one round per nonzero hex digit below 2^20, then powers of two
  const uint32_t *dg = &T.shift[EW_DIG_OFF];
  for (int i = 0; i < 100000; i++) {
    uint64_t n = g() % (1u << 26);
    const uint64_t n0 = n;
    const uint32_t x = g();
    uint32_t y = x;
    for (int p = 0; p < EW_DIG_POS && n; ++p, n >>= 4)
      if (n & 15) y = nib(dg + (p * 15 + (n & 15) - 1) * 128, y);
    y = T.shift_n(n << (4 * EW_DIG_POS), y);
    if (y != T.shift_n(n0, x)) bad++;
  }
  std::printf(bad ? "bad %ld\n" : "ok\n", bad);
  return bad != 0;
}
