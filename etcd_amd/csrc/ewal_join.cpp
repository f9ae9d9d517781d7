// ewal_join.cpp -- ONE WAL read as several ranges: ReadAll's verdict joined
// on the host (ewal_split_verdict), and the one-process multi-context driver
// (ewal_readall_multi) that splits a WAL over several ctxs -- one host thread
// per ctx -- and joins their verdicts.  Plain C++ over the public C ABI
// (include/ewal.h); torch.distributed callers (etcd_amd/shard.py) exchange
// the rows and call the same join.
//
// Reference: (*WAL).ReadAll wal/wal.go:164-216 over MultiReadCloser's
// concatenation of names[nameIndex:] (wal/wal.go:126-134); every file opens
// with crcType{running CRC} (wal/wal.go:93,232-234).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/ewal.h"

namespace {

constexpr uint64_t kNoOp = ~0ull;

// ReadAll over the range ended without a frame of it failing
bool ended_clean(int st) { return st == EWAL_OK || st == EWAL_ERR_INDEX_NOT_FOUND; }

// The metadata bytes of row k inside the md blob: (first, value) as
// (offset, length), length -1 == nil.
struct MdView {
  int64_t first_off = 0, first_len = -1, value_off = 0, value_len = -1;
};

}  // namespace

extern "C" int ewal_split_verdict(const ewal_range_row *rows, uint64_t n, uint64_t ri_global, const uint8_t *md,
                                  uint64_t md_len, ewal_split_result *out) {
  if (!out || (n && !rows)) return EWAL_E_INVAL;
  std::memset(out, 0, sizeof(*out));
  out->fail_record = -1;
  out->resplit = -1;
  // where each row's metadata bytes sit in md
  std::vector<MdView> mv(n);
  uint64_t at = 0;
  for (uint64_t k = 0; k < n; ++k) {
    const ewal_range_info &in = rows[k].info;
    if (in.md_first_frame >= 0 && in.md_first_off >= 0) {
      mv[k].first_off = (int64_t)at;
      mv[k].first_len = in.md_first_len;
      at += (uint64_t)in.md_first_len;
    }
    if (in.md_value_frame >= 0) {
      mv[k].value_off = (int64_t)at;
      mv[k].value_len = in.md_value_len;
      at += (uint64_t)in.md_value_len;
    }
  }
  if (at > md_len || (at && !md)) return EWAL_E_INVAL;
  auto finish = [&](int st, int64_t fail, int64_t frames, int32_t resplit, int64_t detail) {
    out->status = st;
    out->fail_record = fail;
    out->n_records = frames;
    out->resplit = resplit;
    out->detail = detail;
    return EWAL_OK;
  };
  int64_t before = 0;
  uint32_t running = 0;
  bool have_md = false;
  int64_t md_off = 0, md_len_v = 0;        // the metadata value carried (Go's `metadata`)
  uint64_t last_op = kNoOp;                // Index of the last entry op so far (len(ents) - 1 + ri)
  uint64_t enti = 0;
  for (uint64_t k = 0; k < n; ++k) {
    const ewal_range_row &r = rows[k];
    const ewal_range_info &in = r.info;
    if (in.n_bytes == 0) continue;        // an empty range (start == end: joined into an earlier one)
    const int st = r.status;
    const bool failed = !ended_clean(st);
    const int64_t own = failed ? r.fail_record : -1;
    // the first cross-range failure inside this range: (frame, status)
    int64_t cf = -1;
    int cst = 0;
    auto cross = [&](int64_t f, int s) {
      if (cf < 0 || f < cf) { cf = f; cst = s; }
    };
    if (k > 0) {
      if (r.deferred && in.n_frames > 0 && in.first_type != EWAL_CRC) {
        // frame 0's Validate with the running CRC (wal/decoder.go:42-46): only a
        // failure decoder.decode reports before it (framing, Record.Unmarshal) wins
        const uint32_t computed =
            in.first_dlen ? ewal_crc32_combine(0x82F63B78u, running, in.first_u0, in.first_dlen) : running;
        const bool pre = own == 0 && in.first_pre_crc;
        if (computed != in.first_stored_crc && !pre) return finish(EWAL_ERR_RECORD_CRC, before, before, -1, 0);
      } else if (in.first_crc < 0) {
        return finish(st, -1, before, 0, 0);   // its CRCs depend on the range before: verify joined
      }
      // a crcType frame 0 against the running CRC (wal/wal.go:184-192)
      if (in.first_crc >= 0 && running != 0 && (uint32_t)in.first_crc != running) cross(0, EWAL_ERR_WAL_CRC);
      // metadata (wal/wal.go:178-183): metadata != nil && !DeepEqual
      if (have_md && in.md_first_frame >= 0) {
        const bool nil = mv[k].first_len < 0;
        const bool eq = !nil && mv[k].first_len == md_len_v &&
                        std::memcmp(md + mv[k].first_off, md + md_off, (size_t)md_len_v) == 0;
        if (!eq) cross(in.md_first_frame, EWAL_ERR_METADATA_CONFLICT);
      }
      // ents (wal/wal.go:170-173)
      if (in.first_entry_frame >= 0) {
        // entries below the range's w.ri are ops of the whole ReadAll its read skipped
        if (in.min_entry_index < r.ri) return finish(st, -1, before, 0, 0);
        const bool gap_g = last_op != kNoOp ? in.first_entry_index > last_op + 1 : in.first_entry_index > ri_global;
        const bool gap_l = in.first_entry_index > r.ri;
        if (gap_g && !gap_l) cross(in.first_entry_frame, EWAL_PANIC_INDEX_GAP);
        // a gap only the range's read sees hides the rest of the range
        if (gap_l && !gap_g && (own < 0 || own >= in.first_entry_frame)) return finish(st, -1, before, 0, 0);
      }
    }
    // a later range holding bytes: this range's reader would have read on into them
    bool later = false;
    for (uint64_t j = k + 1; j < n; ++j) later = later || rows[j].info.n_bytes > 0;
    if (own >= 0 && (cf < 0 || own <= cf)) {
      // a frame cut short at the range's end reads on into the next range's
      // bytes (MultiReadCloser / one file split): verify joined
      if (st == EWAL_ERR_UNEXPECTED_EOF && later && r.fail_record == r.n_records) {
        out->resplit = (int32_t)k;
        out->status = st;
        out->fail_record = before + own;
        out->n_records = before + own;
        return EWAL_OK;
      }
      return finish(st, before + own, before + own, -1, r.detail);
    }
    if (cf >= 0) return finish(cst, before + cf, before + cf, -1, 0);
    // the range ended short of its last byte (an 8-byte length prefix with no
    // payload reads as io.EOF alone; whole, the stream goes on): verify joined
    if (later && in.end_off != in.n_bytes) return finish(st, -1, before, (int32_t)k, 0);
    before += r.n_records;
    running = r.last_crc;
    if (in.md_value_frame >= 0) {
      have_md = true;
      md_off = mv[k].value_off;
      md_len_v = mv[k].value_len;
    }
    if (in.last_op_frame >= 0) last_op = in.last_op_index;
    if (in.first_entry_frame >= 0) enti = in.last_entry_index;
  }
  out->last_crc = running;
  out->enti = enti;
  if (enti < ri_global) return finish(EWAL_ERR_INDEX_NOT_FOUND, -1, before, -1, 0);
  return finish(EWAL_OK, -1, before, -1, 0);
}

// ---- one process, several contexts ------------------------------------------
namespace {

// A range of the stream read on one ctx.
struct RangeRun {
  uint64_t start = 0, end = 0, ri = 0;
  bool deferred = false;
  ewal_range_row row{};
  std::vector<uint8_t> md;
  int rc = 0;
};

// ReadAll over h[start, end) on ctx (its own device buffer, 16-B aligned),
// the range info and the metadata bytes
void run_range(ewal_ctx *ctx, const uint8_t *h, RangeRun &rr) {
  std::memset(&rr.row, 0, sizeof(rr.row));
  rr.md.clear();
  const uint64_t len = rr.end - rr.start;
  rr.row.ri = rr.ri;
  rr.row.deferred = rr.deferred;
  rr.row.info.n_bytes = len;
  rr.row.info.end_off = len;
  rr.row.info.first_type = -1;
  rr.row.info.first_crc = rr.row.info.md_first_frame = rr.row.info.md_value_frame = -1;
  rr.row.info.first_entry_frame = rr.row.info.last_entry_frame = rr.row.info.last_op_frame = -1;
  rr.row.fail_record = -1;
  if (!len) return;
  void *d = nullptr;
  if ((rr.rc = ewal_device_alloc(ctx, len + 64, &d)) != EWAL_OK) return;
  ewal_result res;
  if ((rr.rc = ewal_upload(ctx, d, h + rr.start, len)) == EWAL_OK) {
    const int st = ewal_readall_range_device(ctx, d, len, rr.ri, rr.deferred ? EWAL_RANGE_DEFER_FIRST : 0u, &res);
    if (st < 0) {
      rr.rc = st;
    } else {
      rr.row.status = res.status;
      rr.row.fail_record = res.fail_record;
      rr.row.n_records = res.n_records;
      rr.row.last_crc = res.last_crc;
      rr.row.detail = res.detail;
      rr.rc = ewal_copy_range_info(ctx, &rr.row.info);
      if (rr.rc == EWAL_OK) {
        const ewal_range_info &in = rr.row.info;
        auto take = [&](int64_t off, int64_t n, bool split) {
          if (split) {   // a metadata Data in several segments: from the ctx's split bytes
            std::vector<uint8_t> all((size_t)std::max<int64_t>(0, ewal_copy_split_bytes(ctx, nullptr, 0)));
            if (!all.empty()) ewal_copy_split_bytes(ctx, all.data(), (int64_t)all.size());
            rr.md.insert(rr.md.end(), all.begin() + off, all.begin() + off + n);
          } else {
            rr.md.insert(rr.md.end(), h + rr.start + off, h + rr.start + off + n);
          }
        };
        if (in.md_first_frame >= 0 && in.md_first_off >= 0) take(in.md_first_off, in.md_first_len, in.md_split & 1);
        if (in.md_value_frame >= 0) take(in.md_value_off, in.md_value_len, in.md_split & 2);
      }
    }
  }
  ewal_device_free(ctx, d);
}

}  // namespace

extern "C" int ewal_readall_multi(ewal_ctx *const *ctxs, uint32_t n_ctx, const void *h_buf, uint64_t len,
                                  const uint64_t *file_off, const uint64_t *file_index, uint32_t n_files, uint64_t ri,
                                  ewal_split_result *out, uint32_t *n_resplit) {
  if (!ctxs || !n_ctx || !out || (len && !h_buf) || (file_off && (!file_index || !n_files))) return EWAL_E_INVAL;
  const uint8_t *h = (const uint8_t *)h_buf;
  const bool by_file = file_off != nullptr;
  if (by_file && (file_off[0] != 0 || file_off[n_files] != len)) return EWAL_E_INVAL;
  std::vector<RangeRun> rr(n_ctx);
  if (by_file) {
    // contiguous runs of whole files, about len / n_ctx bytes each
    uint32_t f = 0;
    for (uint32_t r = 0; r < n_ctx; ++r) {
      const uint32_t f0 = f;
      const uint64_t goal = (uint64_t)((__uint128_t)len * (r + 1) / n_ctx);
      while (f < n_files && (f == f0 || r + 1 == n_ctx || file_off[f] < goal)) ++f;
      rr[r].start = file_off[f0];
      rr[r].end = file_off[f];
      rr[r].ri = (r == 0 || f0 >= n_files) ? ri : std::max(ri, file_index[f0]);
    }
  } else {
    // inside the stream: range r opens at the first frame-start candidate
    // after r * len / n (ewal_range_probe over a window uploaded to ctx r)
    const uint64_t window = 16ull << 20;
    std::vector<int64_t> pos(n_ctx, -1), idx(n_ctx, -1);
    std::vector<int> prc(n_ctx, 0);
    std::vector<std::thread> th;
    for (uint32_t r = 1; r < n_ctx; ++r) {
      th.emplace_back([&, r] {
        const uint64_t from = (uint64_t)((__uint128_t)len * r / n_ctx);
        const uint64_t wl = std::min<uint64_t>(len - from, window);
        if (!wl) return;
        void *d = nullptr;
        if ((prc[r] = ewal_device_alloc(ctxs[r], wl + 64, &d)) != EWAL_OK) return;
        if ((prc[r] = ewal_upload(ctxs[r], d, h + from, wl)) == EWAL_OK) {
          int64_t p = -1, e = -1;
          prc[r] = ewal_range_probe(ctxs[r], d, wl, 0, wl, &p, &e);
          if (prc[r] == EWAL_OK && p >= 0) {
            pos[r] = (int64_t)from + p;
            idx[r] = e;
          }
        }
        ewal_device_free(ctxs[r], d);
      });
    }
    for (auto &t : th) t.join();
    for (uint32_t r = 1; r < n_ctx; ++r)
      if (prc[r] < 0) return prc[r];
    // a share without a candidate gets an empty range: the range before it
    // reaches to the next share's candidate (not to the stream's end)
    std::vector<uint64_t> st(n_ctx + 1, len);
    st[0] = 0;
    for (uint32_t r = n_ctx; r-- > 1;) st[r] = pos[r] >= 0 ? (uint64_t)pos[r] : st[r + 1];
    for (uint32_t r = 1; r < n_ctx; ++r) st[r] = std::max(st[r], st[r - 1]);
    for (uint32_t r = 0; r < n_ctx; ++r) {
      rr[r].start = st[r];
      rr[r].end = st[r + 1];
      rr[r].ri = (r == 0 || idx[r] < 0) ? ri : std::max<uint64_t>(ri, (uint64_t)idx[r]);
      rr[r].deferred = r > 0;
    }
  }
  auto run_all = [&](uint32_t from) {
    std::vector<std::thread> th;
    for (uint32_t r = from; r < n_ctx; ++r) th.emplace_back([&, r] { run_range(ctxs[r], h, rr[r]); });
    for (auto &t : th) t.join();
    for (uint32_t r = from; r < n_ctx; ++r)
      if (rr[r].rc < 0) return rr[r].rc;
    return 0;
  };
  if (int rc = run_all(0)) return rc;
  uint32_t resplits = 0;
  for (;;) {
    std::vector<ewal_range_row> rows(n_ctx);
    std::vector<uint8_t> md;
    for (uint32_t r = 0; r < n_ctx; ++r) {
      rows[r] = rr[r].row;
      md.insert(md.end(), rr[r].md.begin(), rr[r].md.end());
    }
    if (int rc = ewal_split_verdict(rows.data(), n_ctx, ri, md.data(), md.size(), out)) return rc;
    if (out->resplit < 0 || resplits > n_ctx) break;
    // ranges k.. read as one range on ctx k
    const uint32_t k = (uint32_t)out->resplit;
    rr[k].end = len;
    for (uint32_t r = k + 1; r < n_ctx; ++r) rr[r].start = rr[r].end = len;
    ++resplits;
    std::vector<std::thread> th;
    for (uint32_t r = k; r < n_ctx; ++r) th.emplace_back([&, r] { run_range(ctxs[r], h, rr[r]); });
    for (auto &t : th) t.join();
    for (uint32_t r = k; r < n_ctx; ++r)
      if (rr[r].rc < 0) return rr[r].rc;
  }
  if (n_resplit) *n_resplit = resplits;
  return EWAL_OK;
}
