// san_join.cpp -- ASan + UBSan driver of the host-only join of ONE WAL read as
// several ranges (etcd_amd/csrc/ewal_join.cpp: ewal_split_verdict and
// ewal_split_ents_layout), over rows tests/test_sanitizers.py built from the
// oracle's per-range ReadAll + range info (by-file splits of clean, corrupt,
// torn, seam, metadata, index-rule and mutated WALs; resplits followed).
//
// Input file: repeated cases of
//   u64 n, u64 ri_global, u64 md_len, md bytes, n x ewal_range_row (raw)
// Output: one line per case:
//   status fail_record n_records resplit last_crc enti md_range md_blob_off md_len state_range n_ents
//   | layout: base:count per range (only for a final EWAL_OK)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ewal.h"

static bool rd(FILE *f, void *p, size_t n) { return std::fread(p, 1, n, f) == n; }

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int cases = 0;
  for (;;) {
    uint64_t n = 0, rig = 0, mdl = 0;
    if (!rd(f, &n, 8)) break;
    if (!rd(f, &rig, 8) || !rd(f, &mdl, 8)) return 3;
    // exact-size heap buffers, so an overrun of either is an ASan report
    std::vector<uint8_t> md(mdl);
    if (mdl && !rd(f, md.data(), mdl)) return 3;
    std::vector<ewal_range_row> rows(n);
    if (n && !rd(f, rows.data(), n * sizeof(ewal_range_row))) return 3;
    ewal_split_result out;
    const int rc = ewal_split_verdict(n ? rows.data() : nullptr, n, rig, mdl ? md.data() : nullptr, mdl, &out);
    if (rc) {
      std::printf("rc %d\n", rc);
      ++cases;
      continue;
    }
    std::printf("%d %lld %lld %d %u %llu %d %lld %lld %d %lld |", out.status, (long long)out.fail_record,
                (long long)out.n_records, out.resplit, (unsigned)out.last_crc, (unsigned long long)out.enti,
                out.md_range, (long long)out.md_blob_off, (long long)out.md_len, out.state_range,
                (long long)out.n_ents);
    if (out.status == EWAL_OK && out.resplit < 0) {
      std::vector<int64_t> base(n), count(n);
      const int64_t len = ewal_split_ents_layout(rows.data(), n, rig, base.data(), count.data());
      std::printf(" %lld", (long long)len);
      for (uint64_t k = 0; k < n; ++k) std::printf(" %lld:%lld", (long long)base[k], (long long)count[k]);
    }
    std::printf("\n");
    ++cases;
  }
  std::fclose(f);
  std::fprintf(stderr, "san_join ok (%d cases)\n", cases);
  return 0;
}
