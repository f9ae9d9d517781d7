// crc_math.h -- reflected CRC-32 arithmetic used by the engine (host side).
//
// Restates Go hash/crc32 (Update(crc, tab, p) = ^update(^crc, tab, p); the
// call sites are pkg/crc/crc.go:32, snap/snapshotter.go:53,98, wal/wal.go:49)
// in the affine form the GPU pipeline needs:
//
//   raw(c, D)        register after feeding D from register c (no inversion)
//   lin(D)           raw(0, D)                       -- GF(2)-linear in D
//   S_n(c)           raw(c, n zero bytes)            -- GF(2)-linear in c
//   raw(c, A||B)   = S_|B|(raw(c, A)) ^ lin(B)
//   Update(c, D)   = S_n(c ^ ~0) ^ lin(D) ^ ~0 = S_n(c) ^ Update(0, D)
//
// Tables built here (per polynomial) and uploaded to the device:
//   slice[4][256]      slicing-by-4 tables (slice[0] = MakeTable(poly))
//   shift[m][4][256]   byte tables of S_{2^m}, m = 0..EW_SHIFT_LEVELS-1:
//                      S_{2^m}(x) = ^_k shift[m][k][(x >> 8k) & 0xff];
//                      then EW_INV_LEVELS more: the inverses S_{2^m}^-1
//                      (S_1 is x -> x * x^8 mod the polynomial, invertible
//                      because the polynomial has a constant term), so that
//                      P(x) = S_{b-x}^-1(P(b) ^ lin(stream[x, b))) reaches a
//                      prefix from the NEXT boundary b;
//                      then EW_TAIL_TABS nibble tables (128 words each) of
//                      the shifts by -128..128 bytes in two factors, for the
//                      frame pass's prefix tails (tail_shift in
//                      wal_kernels.hip): S_{16a} (a = 0..8), S_b (b = 0..15),
//                      S_{16a}^-1, S_b^-1; then S_{16a} (a = 9..15) and
//                      S_{256a} (a = 1..15), with which the checks take the
//                      low 12 bits of S_dlen in three rounds (frame_kernels.hip);
//                      then EW_DIG_TABS digit tables S_{d 16^p} for the seam
//                      pass's shifts by n < 2^20 in <= 5 rounds (seam_shift)
#pragma once
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#define EW_SHIFT_LEVELS 48  // S_{2^m} for m < 48: lengths up to 256 TiB
#define EW_INV_LEVELS 8     // S_{2^m}^-1 for m < 8 (inverse shifts up to 255 bytes), after the forward levels
#define EW_TAIL_TABS 72     // nibble tables after the inverse levels (see above); then S_{16a} (a = 9..15)
                            // and S_{256a} (a = 1..15) for the checks' S_dlen
#define EW_TAIL_OFF ((EW_SHIFT_LEVELS + EW_INV_LEVELS) * 1024)
#define EW_DIG_POS 5        // then digit tables for the seam pass: S_{d 16^p}, p < EW_DIG_POS, d = 1..15
#define EW_DIG_OFF (EW_TAIL_OFF + EW_TAIL_TABS * 128)
#define EW_DIG_TABS (EW_DIG_POS * 15)

// The signed shift amount of tail table t: S_{16t}, S_{t-9}, S_{16(t-25)}^-1, S_{t-34}^-1, S_{16(t-41)},
// S_{256(t-56)}
inline int ew_tail_amount(int t) {
  return t < 9 ? 16 * t : t < 25 ? t - 9 : t < 34 ? -16 * (t - 25) : t < 50 ? -(t - 34) : t < 57 ? 16 * (t - 41) : 256 * (t - 56);
}

namespace ewal {

struct CrcTables {
  uint32_t poly = 0;
  uint32_t slice[4][256];
  uint32_t slice16[16][256];    // slicing-by-16 (slice16[t] = slice[t] for t < 4): the device table
  std::vector<uint32_t> shift;  // EW_SHIFT_LEVELS * 4 * 256

  explicit CrcTables(uint32_t p) : poly(p), shift((size_t)EW_DIG_OFF + EW_DIG_TABS * 128) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
      slice[0][i] = c;
    }
    for (int t = 1; t < 4; t++)
      for (uint32_t i = 0; i < 256; i++)
        slice[t][i] = (slice[t - 1][i] >> 8) ^ slice[0][slice[t - 1][i] & 0xff];
    std::memcpy(slice16, slice, sizeof(slice));
    for (int t = 4; t < 16; t++)
      for (uint32_t i = 0; i < 256; i++)
        slice16[t][i] = (slice16[t - 1][i] >> 8) ^ slice[0][slice16[t - 1][i] & 0xff];
    // S_1 as a GF(2) matrix (column j = S_1(1 << j)), then repeated squaring.
    uint32_t m[32], sq[32];
    for (int j = 0; j < 32; j++) {
      uint32_t x = 1u << j;
      m[j] = slice[0][x & 0xff] ^ (x >> 8);
    }
    uint32_t m1[32];
    std::memcpy(m1, m, sizeof(m1));
    for (int lvl = 0; lvl < EW_SHIFT_LEVELS; lvl++) {
      uint32_t *tb = &shift[(size_t)lvl * 1024];
      for (int k = 0; k < 4; k++)
        for (uint32_t b = 0; b < 256; b++) tb[k * 256 + b] = matvec(m, b << (8 * k));
      for (int j = 0; j < 32; j++) sq[j] = matvec(m, m[j]);
      std::memcpy(m, sq, sizeof(m));
    }
    // S_1^-1 by Gauss-Jordan over GF(2), then its powers S_{2^m}^-1
    invert(m1, m);
    for (int lvl = 0; lvl < EW_INV_LEVELS; lvl++) {
      uint32_t *tb = &shift[(size_t)(EW_SHIFT_LEVELS + lvl) * 1024];
      for (int k = 0; k < 4; k++)
        for (uint32_t b = 0; b < 256; b++) tb[k * 256 + b] = matvec(m, b << (8 * k));
      for (int j = 0; j < 32; j++) sq[j] = matvec(m, m[j]);
      std::memcpy(m, sq, sizeof(m));
    }
    for (int t = 0; t < EW_TAIL_TABS; t++) {
      const int a = ew_tail_amount(t);
      for (int k = 0; k < 8; k++)
        for (uint32_t d = 0; d < 16; d++) shift[(size_t)EW_TAIL_OFF + t * 128 + k * 16 + d] = shift_signed(a, d << (4 * k));
    }
    for (int t = 0; t < EW_DIG_TABS; t++) {
      const uint64_t n = (uint64_t)(t % 15 + 1) << (4 * (t / 15));
      for (int k = 0; k < 8; k++)
        for (uint32_t d = 0; d < 16; d++) shift[(size_t)EW_DIG_OFF + t * 128 + k * 16 + d] = shift_n(n, d << (4 * k));
    }
  }

  // inverse of the GF(2) matrix a (column j = a[j]) into r
  static void invert(const uint32_t *a, uint32_t *r) {
    // rows of [A | I]: row i holds bit i of every column
    uint32_t ra[32], ri[32];
    for (int i = 0; i < 32; i++) {
      ra[i] = 0;
      ri[i] = 1u << i;
      for (int j = 0; j < 32; j++) ra[i] |= ((a[j] >> i) & 1u) << j;
    }
    for (int c = 0; c < 32; c++) {
      int piv = c;
      while (piv < 32 && !((ra[piv] >> c) & 1u)) piv++;
      if (piv == 32) return;   // singular (not for a CRC polynomial with a constant term)
      std::swap(ra[c], ra[piv]);
      std::swap(ri[c], ri[piv]);
      for (int i = 0; i < 32; i++)
        if (i != c && ((ra[i] >> c) & 1u)) { ra[i] ^= ra[c]; ri[i] ^= ri[c]; }
    }
    // ri row i = row i of A^-1; back to columns
    for (int j = 0; j < 32; j++) {
      r[j] = 0;
      for (int i = 0; i < 32; i++) r[j] |= ((ri[i] >> j) & 1u) << i;
    }
  }

  static uint32_t matvec(const uint32_t *m, uint32_t x) {
    uint32_t r = 0;
    for (int j = 0; x; j++, x >>= 1)
      if (x & 1) r ^= m[j];
    return r;
  }

  uint32_t shift_pow2(int lvl, uint32_t x) const {
    const uint32_t *tb = &shift[(size_t)lvl * 1024];
    return tb[x & 0xff] ^ tb[256 + ((x >> 8) & 0xff)] ^ tb[512 + ((x >> 16) & 0xff)] ^ tb[768 + (x >> 24)];
  }
  // S_n(x) for -256 < n < 2^48 (negative: the inverse levels)
  uint32_t shift_signed(int64_t n, uint32_t x) const {
    if (n >= 0) return shift_n((uint64_t)n, x);
    for (int lvl = 0, u = (int)-n; u; lvl++, u >>= 1)
      if (u & 1) x = shift_pow2(EW_SHIFT_LEVELS + lvl, x);
    return x;
  }
  // S_n(x) for any n < 2^48.
  uint32_t shift_n(uint64_t n, uint32_t x) const {
    for (int lvl = 0; n; lvl++, n >>= 1)
      if (n & 1) x = shift_pow2(lvl, x);
    return x;
  }
  uint32_t raw(uint32_t c, const uint8_t *p, size_t n) const {
    while (n >= 4) {
      uint32_t w;
      std::memcpy(&w, p, 4);
      c ^= w;
      c = slice[3][c & 0xff] ^ slice[2][(c >> 8) & 0xff] ^ slice[1][(c >> 16) & 0xff] ^ slice[0][c >> 24];
      p += 4;
      n -= 4;
    }
    while (n--) c = slice[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    return c;
  }
  uint32_t update(uint32_t crc, const uint8_t *p, size_t n) const { return ~raw(~crc, p, n); }
  // Update(crc_a, B) given crc_b = Update(0, B): S_n(crc_a) ^ crc_b.
  uint32_t combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) const { return shift_n(len_b, crc_a) ^ crc_b; }
};

}  // namespace ewal
