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
#include <chrono>
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
  out->md_range = out->state_range = -1;
  out->md_off = out->md_blob_off = 0;
  out->md_len = -1;
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
    if (in.md_value_frame >= 0 && !have_md) {   // the value ReadAll returns: the first non-nil Data
      have_md = true;
      md_off = mv[k].value_off;
      md_len_v = mv[k].value_len;
      out->md_range = (int32_t)k;
      out->md_split = (in.md_split & 2) ? 1 : 0;
      out->md_off = in.md_value_off;
      out->md_len = in.md_value_len;
      out->md_blob_off = md_off;
    }
    if (in.state_frame >= 0) {   // state = mustUnmarshalState(rec.Data): the last one wins
      out->state_range = (int32_t)k;
      out->state_term = in.state_term;
      out->state_vote = in.state_vote;
      out->state_commit = in.state_commit;
    }
    if (in.last_op_frame >= 0) last_op = in.last_op_index;
    if (in.first_entry_frame >= 0) enti = in.last_entry_index;
  }
  out->last_crc = running;
  out->enti = enti;
  if (enti < ri_global) {
    out->md_range = out->state_range = -1;
    out->md_len = -1;
    return finish(EWAL_ERR_INDEX_NOT_FOUND, -1, before, -1, 0);
  }
  // a HardState with unknown fields from a range whose own ReadAll kept no
  // side list (its status was not EWAL_OK: ErrIndexNotFound, a range with no
  // entry op at or past its w.ri -- e.g. a last file of crc + metadata +
  // HardState after a Cut).  Re-reading from that range on gives the same
  // status again when it is the last range holding bytes, so the
  // ranges are read joined from the last EARLIER range whose own ReadAll ended
  // EWAL_OK (its entries carry the joined read's enti to its w.ri), else from
  // range 0 (the whole ReadAll, whose verdict this one is).  Every such resplit
  // moves strictly earlier, so the caller's re-reads end.
  if (out->state_range >= 0) {
    const ewal_range_row &r = rows[out->state_range];
    if (r.info.state_unrec && r.status != EWAL_OK) {
      int32_t k = 0;
      for (int32_t j = out->state_range - 1; j > 0; --j)
        if (rows[j].info.n_bytes && rows[j].status == EWAL_OK) {
          k = j;
          break;
        }
      return finish(EWAL_OK, -1, before, k, 0);
    }
  }
  out->n_ents = ewal_split_ents_layout(rows, n, ri_global, nullptr, nullptr);
  return finish(EWAL_OK, -1, before, -1, 0);
}

extern "C" int64_t ewal_split_ents_layout(const ewal_range_row *rows, uint64_t n, uint64_t ri_global, int64_t *base,
                                          int64_t *count) {
  if (n && !rows) return EWAL_E_INVAL;
  int64_t len = 0;
  for (uint64_t k = 0; k < n; ++k) {
    const ewal_range_info &in = rows[k].info;
    int64_t b = 0, c = 0;
    if (in.n_bytes && in.last_op_frame >= 0 && in.last_op_index >= rows[k].ri && rows[k].ri >= ri_global) {
      b = (int64_t)(rows[k].ri - ri_global);
      c = (int64_t)(in.last_op_index - rows[k].ri + 1);
      if (b > len) return EWAL_E_INVAL;   // a gap the verdict reports (never a final EWAL_OK)
      // ents = append(ents[:Index - ri], e): the earlier ranges' ents at or past b are overwritten
      if (count)
        for (uint64_t j = 0; j < k; ++j)
          if (count[j] > 0 && base[j] + count[j] > b) count[j] = std::max<int64_t>(0, b - base[j]);
      len = b + c;
    }
    if (base) base[k] = b;
    if (count) count[k] = c;
  }
  return len;
}

// ---- one process, several contexts ------------------------------------------
namespace {

// A range of the stream read on one ctx.
struct RangeRun {
  uint64_t start = 0, end = 0, ri = 0;
  bool deferred = false;
  const uint8_t *dev = nullptr;   // device-resident: the range's bytes on its ctx (nullptr: staged from host)
  ewal_range_row row{};
  std::vector<uint8_t> md;
  double ms = 0;                  // device time of the range's ReadAll
  int rc = 0;
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// The joined ReadAll of one WAL over several contexts (ewal_multi_*).
struct ewal_multi {
  std::vector<ewal_ctx *> ctxs;
  std::vector<RangeRun> rr;       // the last call's ranges, in stream order
  const uint8_t *h = nullptr;     // the last host call's bytes
  uint64_t len = 0, ri = 0;
  ewal_split_result res{};
  bool valid = false;             // res is a final verdict of the last call
  uint32_t resplits = 0;
  double wall_ms = 0, join_ms = 0;
  // lazily built joined side data
  bool split_done = false, unrec_done = false;
  std::vector<int64_t> split_base;   // per range: its split bytes' offset in the joined split bytes
  std::vector<uint8_t> split;        // the joined split bytes
  std::vector<ewal_unrec> unrec;
  std::vector<uint8_t> unrec_bytes;
};

namespace {

void row_init(RangeRun &rr) {
  std::memset(&rr.row, 0, sizeof(rr.row));
  rr.md.clear();
  rr.ms = 0;
  rr.rc = 0;
  const uint64_t len = rr.end - rr.start;
  rr.row.ri = rr.ri;
  rr.row.deferred = rr.deferred;
  rr.row.info.n_bytes = len;
  rr.row.info.end_off = len;
  rr.row.info.first_type = -1;
  rr.row.info.first_crc = rr.row.info.md_first_frame = rr.row.info.md_value_frame = -1;
  rr.row.info.first_entry_frame = rr.row.info.last_entry_frame = rr.row.info.last_op_frame = -1;
  rr.row.info.state_frame = -1;
  rr.row.fail_record = -1;
}

// ReadAll over the range on ctx (its bytes device-resident at rr.dev, or
// h[start, end) staged into the ctx's reusable staging buffer), the range
// info and the metadata bytes
void run_range(ewal_ctx *ctx, const uint8_t *h, RangeRun &rr) {
  row_init(rr);
  const uint64_t len = rr.end - rr.start;
  if (!len) return;
  const uint8_t *d = rr.dev;
  if (!d) {
    void *s = nullptr;
    if ((rr.rc = ewal_stage_to_device(ctx, h + rr.start, len, &s)) != EWAL_OK) return;
    d = (const uint8_t *)s;
  }
  ewal_result res;
  const int st = ewal_readall_range_device(ctx, d, len, rr.ri, rr.deferred ? EWAL_RANGE_DEFER_FIRST : 0u, &res);
  if (st < 0) {
    rr.rc = st;
    return;
  }
  rr.ms = res.device_ms;
  rr.row.status = res.status;
  rr.row.fail_record = res.fail_record;
  rr.row.n_records = res.n_records;
  rr.row.last_crc = res.last_crc;
  rr.row.detail = res.detail;
  if ((rr.rc = ewal_copy_range_info(ctx, &rr.row.info)) != EWAL_OK) return;
  const ewal_range_info &in = rr.row.info;
  auto take = [&](int64_t off, int64_t n, bool split) {
    if (n <= 0) return;
    const size_t at = rr.md.size();
    if (split) {   // a metadata Data in several segments: from the ctx's split bytes
      std::vector<uint8_t> all((size_t)std::max<int64_t>(0, ewal_copy_split_bytes(ctx, nullptr, 0)));
      if (!all.empty()) ewal_copy_split_bytes(ctx, all.data(), (int64_t)all.size());
      rr.md.insert(rr.md.end(), all.begin() + off, all.begin() + off + n);
    } else if (!rr.dev) {
      rr.md.insert(rr.md.end(), h + rr.start + off, h + rr.start + off + n);
    } else {
      rr.md.resize(at + (size_t)n);
      if (int rc = ewal_download(ctx, rr.md.data() + at, d + off, (uint64_t)n)) rr.rc = rc;
    }
  };
  if (in.md_first_frame >= 0 && in.md_first_off >= 0) take(in.md_first_off, in.md_first_len, in.md_split & 1);
  if (in.md_value_frame >= 0) take(in.md_value_off, in.md_value_len, in.md_split & 2);
}

int run_ranges(ewal_multi *m, uint32_t from) {
  std::vector<std::thread> th;
  for (uint32_t r = from; r < m->ctxs.size(); ++r) th.emplace_back([m, r] { run_range(m->ctxs[r], m->h, m->rr[r]); });
  for (auto &t : th) t.join();
  for (uint32_t r = from; r < m->ctxs.size(); ++r)
    if (m->rr[r].rc < 0) return m->rr[r].rc;
  return 0;
}

// Join the ranges; re-read ranges k.. joined on ctx k while the verdict asks
// (host bytes: staged again; device-resident: only when ranges k.. are one
// contiguous device span, else the verdict is handed back with resplit = k).
int join_ranges(ewal_multi *m, ewal_split_result *out) {
  const uint32_t n = (uint32_t)m->ctxs.size();
  m->resplits = 0;
  for (;;) {
    const double t0 = now_ms();
    std::vector<ewal_range_row> rows(n);
    std::vector<uint8_t> md;
    for (uint32_t r = 0; r < n; ++r) {
      rows[r] = m->rr[r].row;
      md.insert(md.end(), m->rr[r].md.begin(), m->rr[r].md.end());
    }
    const int rc = ewal_split_verdict(rows.data(), n, m->ri, md.data(), md.size(), out);
    m->join_ms += now_ms() - t0;
    if (rc) return rc;
    if (out->resplit < 0) break;
    // every resplit moves to an earlier range or reads the rest as one, so
    // more than n of them means the verdict never settled: an internal error
    if (m->resplits > n) return EWAL_E_INVAL;
    const uint32_t k = (uint32_t)out->resplit;
    if (m->rr[k].dev) {
      for (uint32_t r = k; r + 1 < n; ++r)
        if (m->rr[r + 1].end > m->rr[r + 1].start && m->rr[r].dev + (m->rr[r].end - m->rr[r].start) != m->rr[r + 1].dev)
          return EWAL_OK;   // not one device span: the caller reads ranges k.. joined
    }
    m->rr[k].end = m->len;
    for (uint32_t r = k + 1; r < n; ++r) {
      m->rr[r].start = m->rr[r].end = m->len;
      m->rr[r].dev = nullptr;
    }
    ++m->resplits;
    if (int rc2 = run_ranges(m, k)) return rc2;
  }
  return EWAL_OK;
}

int check_ctxs(ewal_ctx *const *ctxs, uint32_t n) {
  if (!ctxs || !n) return EWAL_E_INVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (!ctxs[i]) return EWAL_E_INVAL;
    for (uint32_t j = 0; j < i; ++j)
      if (ctxs[j] == ctxs[i]) return EWAL_E_INVAL;   // one ctx is never driven from two threads
  }
  return EWAL_OK;
}

void reset_call(ewal_multi *m) {
  m->valid = false;
  m->split_done = m->unrec_done = false;
  m->split.clear();
  m->split_base.clear();
  m->unrec.clear();
  m->unrec_bytes.clear();
  m->join_ms = 0;
  m->resplits = 0;
}

}  // namespace

extern "C" int ewal_multi_create(ewal_ctx *const *ctxs, uint32_t n_ctx, ewal_multi **out) {
  if (!out) return EWAL_E_INVAL;
  *out = nullptr;
  if (int rc = check_ctxs(ctxs, n_ctx)) return rc;
  ewal_multi *m = new ewal_multi;
  m->ctxs.assign(ctxs, ctxs + n_ctx);
  m->rr.resize(n_ctx);
  *out = m;
  return EWAL_OK;
}

extern "C" void ewal_multi_destroy(ewal_multi *m) { delete m; }

extern "C" int ewal_multi_readall(ewal_multi *m, const void *h_buf, uint64_t len, const uint64_t *file_off,
                                  const uint64_t *file_index, uint32_t n_files, uint64_t ri, ewal_split_result *out) {
  if (!m || !out || (len && !h_buf) || (file_off && (!file_index || !n_files))) return EWAL_E_INVAL;
  const double t0 = now_ms();
  reset_call(m);
  const uint32_t n_ctx = (uint32_t)m->ctxs.size();
  const uint8_t *h = (const uint8_t *)h_buf;
  const bool by_file = file_off != nullptr;
  if (by_file && (file_off[0] != 0 || file_off[n_files] != len)) return EWAL_E_INVAL;
  m->h = h;
  m->len = len;
  m->ri = ri;
  std::vector<RangeRun> &rr = m->rr;
  for (RangeRun &x : rr) x = RangeRun();
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
    // after r * len / n (ewal_range_probe over a window staged on ctx r)
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
        if ((prc[r] = ewal_stage_to_device(m->ctxs[r], h + from, wl, &d)) != EWAL_OK) return;
        int64_t p = -1, e = -1;
        prc[r] = ewal_range_probe(m->ctxs[r], d, wl, 0, wl, &p, &e);
        if (prc[r] == EWAL_OK && p >= 0) {
          pos[r] = (int64_t)from + p;
          idx[r] = e;
        }
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
  if (int rc = run_ranges(m, 0)) return rc;
  if (int rc = join_ranges(m, out)) return rc;
  m->res = *out;
  m->valid = out->resplit < 0;
  m->wall_ms = now_ms() - t0;
  return EWAL_OK;
}

extern "C" int ewal_multi_plan_device(ewal_multi *m, const void *d_buf, uint64_t len, uint64_t ri, uint64_t *starts,
                                      uint64_t *ris) {
  if (!m || !starts || !ris || (len && !d_buf)) return EWAL_E_INVAL;
  const uint32_t n_ctx = (uint32_t)m->ctxs.size();
  const uint8_t *d = (const uint8_t *)d_buf;
  std::vector<int64_t> pos(n_ctx, -1), idx(n_ctx, -1);
  std::vector<int> prc(n_ctx, 0);
  std::vector<std::thread> th;
  for (uint32_t r = 1; r < n_ctx; ++r) {
    th.emplace_back([&, r] {
      // a 16-B aligned frame-start candidate after r * len / n (the range's
      // bytes then start on an aligned address: no copy: ewal_readall_device
      // reads 16-B aligned buffers only).  A window of 64 MiB with no aligned
      // candidate (entries that large) leaves range r EMPTY: its start is the
      // next range's, so the previous range reads on through it -- visible to
      // the caller as starts[r] == starts[r + 1] in the plan (unbalanced, never
      // wrong).
      const uint64_t from = (uint64_t)((__uint128_t)len * r / n_ctx);
      const uint64_t wl = std::min<uint64_t>(len - from, 64ull << 20);
      if (!wl) return;
      int64_t p = -1, e = -1;
      prc[r] = ewal_range_probe_aligned(m->ctxs[r], d, len, from, wl, 16, &p, &e);
      if (prc[r] == EWAL_OK && p >= 0) {
        pos[r] = p;
        idx[r] = e;
      }
    });
  }
  for (auto &t : th) t.join();
  for (uint32_t r = 1; r < n_ctx; ++r)
    if (prc[r] < 0) return prc[r];
  std::vector<uint64_t> st(n_ctx + 1, len);
  st[0] = 0;
  for (uint32_t r = n_ctx; r-- > 1;) st[r] = pos[r] >= 0 ? (uint64_t)pos[r] : st[r + 1];
  for (uint32_t r = 1; r < n_ctx; ++r) st[r] = std::max(st[r], st[r - 1]);
  for (uint32_t r = 0; r < n_ctx; ++r) {
    starts[r] = st[r];
    ris[r] = (r == 0 || idx[r] < 0) ? ri : std::max<uint64_t>(ri, (uint64_t)idx[r]);
  }
  starts[n_ctx] = len;
  return EWAL_OK;
}

extern "C" int ewal_multi_readall_device(ewal_multi *m, const void *const *d_ranges, const uint64_t *starts,
                                         const uint64_t *ris, const uint32_t *flags, uint64_t ri,
                                         ewal_split_result *out) {
  if (!m || !out || !d_ranges || !starts || !ris) return EWAL_E_INVAL;
  const double t0 = now_ms();
  reset_call(m);
  const uint32_t n_ctx = (uint32_t)m->ctxs.size();
  if (starts[0] != 0) return EWAL_E_INVAL;
  for (uint32_t r = 0; r < n_ctx; ++r) {
    if (starts[r + 1] < starts[r]) return EWAL_E_INVAL;
    if (starts[r + 1] > starts[r] && (!d_ranges[r] || ((uintptr_t)d_ranges[r] & 15))) return EWAL_E_INVAL;
  }
  m->h = nullptr;
  m->len = starts[n_ctx];
  m->ri = ri;
  for (uint32_t r = 0; r < n_ctx; ++r) {
    RangeRun &x = m->rr[r];
    x = RangeRun();
    x.start = starts[r];
    x.end = starts[r + 1];
    x.ri = ris[r];
    x.deferred = flags ? (flags[r] & EWAL_RANGE_DEFER_FIRST) != 0 : r > 0;
    x.dev = (const uint8_t *)d_ranges[r];
  }
  if (int rc = run_ranges(m, 0)) return rc;
  if (int rc = join_ranges(m, out)) return rc;
  m->res = *out;
  m->valid = out->resplit < 0;
  m->wall_ms = now_ms() - t0;
  return EWAL_OK;
}

extern "C" int ewal_multi_timing(ewal_multi *m, double *out4) {
  if (!m || !out4) return EWAL_E_INVAL;
  double dmax = 0;
  for (const RangeRun &x : m->rr) dmax = std::max(dmax, x.ms);
  out4[0] = m->wall_ms;
  out4[1] = dmax;
  out4[2] = m->join_ms;
  out4[3] = (double)m->resplits;
  return EWAL_OK;
}

extern "C" int ewal_multi_copy_rows(ewal_multi *m, ewal_range_row *out, uint64_t *starts, uint32_t cap) {
  if (!m || (cap && (!out || !starts))) return EWAL_E_INVAL;
  const uint32_t n = (uint32_t)std::min<size_t>(cap, m->rr.size());
  for (uint32_t r = 0; r < n; ++r) {
    out[r] = m->rr[r].row;
    starts[r] = m->rr[r].start;
  }
  return (int)m->rr.size();
}

namespace {

// the joined split bytes: every range's, in order
int build_split(ewal_multi *m) {
  if (m->split_done) return EWAL_OK;
  m->split.clear();
  m->split_base.assign(m->rr.size(), 0);
  for (size_t r = 0; r < m->rr.size(); ++r) {
    m->split_base[r] = (int64_t)m->split.size();
    if (m->rr[r].end == m->rr[r].start) continue;
    const int64_t n = ewal_copy_split_bytes(m->ctxs[r], nullptr, 0);
    if (n < 0) return (int)n;
    if (!n) continue;
    const size_t at = m->split.size();
    m->split.resize(at + (size_t)n);
    const int64_t got = ewal_copy_split_bytes(m->ctxs[r], m->split.data() + at, n);
    if (got < 0) return (int)got;
  }
  m->split_done = true;
  return EWAL_OK;
}

std::vector<ewal_range_row> rows_of(const ewal_multi *m) {
  std::vector<ewal_range_row> rows(m->rr.size());
  for (size_t r = 0; r < rows.size(); ++r) rows[r] = m->rr[r].row;
  return rows;
}

}  // namespace

extern "C" int64_t ewal_multi_copy_entries(ewal_multi *m, ewal_entry *out, int64_t cap) {
  if (!m || (!out && cap) || cap < 0) return EWAL_E_INVAL;
  if (!m->valid || m->res.status != EWAL_OK) return 0;
  const std::vector<ewal_range_row> rows = rows_of(m);
  const size_t n = rows.size();
  std::vector<int64_t> base(n), count(n);
  const int64_t total = ewal_split_ents_layout(rows.data(), n, m->ri, base.data(), count.data());
  if (total < 0) return total;
  if (int rc = build_split(m)) return rc;
  std::vector<ewal_entry> tmp;
  for (size_t r = 0; r < n; ++r) {
    if (count[r] <= 0 || base[r] >= cap) continue;
    const int64_t want = std::min<int64_t>(count[r], cap - base[r]);
    tmp.resize((size_t)want);
    const int64_t got = ewal_copy_entries(m->ctxs[r], tmp.data(), want);
    if (got < 0) return got;
    if (got != want) return EWAL_E_INVAL;   // the ctx no longer holds that range's ReadAll
    for (int64_t j = 0; j < got; ++j) {
      ewal_entry e = tmp[(size_t)j];
      // Data views into the whole stream (split Data: into the joined split bytes)
      e.data_off += e.data_nil == 2 ? (uint64_t)m->split_base[r] : m->rr[r].start;
      out[base[r] + j] = e;
    }
  }
  return std::min<int64_t>(total, cap);
}

extern "C" int64_t ewal_multi_copy_split_bytes(ewal_multi *m, uint8_t *out, int64_t cap) {
  if (!m || (!out && cap) || cap < 0) return EWAL_E_INVAL;
  if (!m->valid || m->res.status != EWAL_OK) return 0;
  if (int rc = build_split(m)) return rc;
  const int64_t n = std::min<int64_t>(cap, (int64_t)m->split.size());
  if (n > 0) std::memcpy(out, m->split.data(), (size_t)n);
  return (int64_t)m->split.size();
}

extern "C" int64_t ewal_multi_copy_metadata(ewal_multi *m, uint8_t *out, int64_t cap) {
  if (!m || (!out && cap) || cap < 0) return EWAL_E_INVAL;
  if (!m->valid || m->res.status != EWAL_OK || m->res.md_range < 0) return 0;
  const RangeRun &x = m->rr[(size_t)m->res.md_range];
  // the range's metadata bytes: [first's Data][value's Data]; the value is last
  const int64_t len = m->res.md_len;
  if (len <= 0 || (int64_t)x.md.size() < len) return len < 0 ? 0 : len;
  const int64_t n = std::min<int64_t>(cap, len);
  if (n > 0) std::memcpy(out, x.md.data() + (x.md.size() - (size_t)len), (size_t)n);
  return len;
}

namespace {

int build_unrec(ewal_multi *m) {
  if (m->unrec_done) return EWAL_OK;
  m->unrec.clear();
  m->unrec_bytes.clear();
  const std::vector<ewal_range_row> rows = rows_of(m);
  const size_t n = rows.size();
  std::vector<int64_t> base(n), count(n);
  if (ewal_split_ents_layout(rows.data(), n, m->ri, base.data(), count.data()) < 0) return EWAL_E_INVAL;
  for (size_t r = 0; r < n; ++r) {
    const bool st_here = m->res.state_range == (int32_t)r && rows[r].info.state_unrec;
    if (count[r] <= 0 && !st_here) continue;
    if (rows[r].status != EWAL_OK) continue;   // (no entry ops there; a state with unknown fields was re-read joined)
    // (ewal_copy_unrec returns the number copied: ask with a growing cap)
    std::vector<ewal_unrec> u;
    int64_t cap = 64;
    for (;;) {
      u.resize((size_t)cap);
      const int64_t got = ewal_copy_unrec(m->ctxs[r], u.data(), cap);
      if (got < 0) return (int)got;
      if (got < cap) {
        u.resize((size_t)got);
        break;
      }
      cap *= 2;
    }
    if (u.empty()) continue;
    uint64_t nb = 0;
    for (const ewal_unrec &x : u) nb = std::max<uint64_t>(nb, x.off + x.len);
    std::vector<uint8_t> b((size_t)nb);
    if (nb) {
      const int64_t got = ewal_copy_unrec_bytes(m->ctxs[r], b.data(), (int64_t)nb);
      if (got < 0) return (int)got;
    }
    for (const ewal_unrec &x : u) {
      const bool keep = x.ent < 0 ? st_here : x.ent < count[r];
      if (!keep) continue;
      ewal_unrec y = x;
      y.ent = x.ent < 0 ? -1 : base[r] + x.ent;
      y.off = m->unrec_bytes.size();
      m->unrec_bytes.insert(m->unrec_bytes.end(), b.begin() + x.off, b.begin() + x.off + x.len);
      m->unrec.push_back(y);
    }
  }
  std::stable_sort(m->unrec.begin(), m->unrec.end(), [](const ewal_unrec &a, const ewal_unrec &b) {
    return (uint64_t)a.ent < (uint64_t)b.ent;   // ents in order, the HardState (-1) last
  });
  m->unrec_done = true;
  return EWAL_OK;
}

}  // namespace

extern "C" int64_t ewal_multi_copy_unrec(ewal_multi *m, ewal_unrec *out, int64_t cap) {
  if (!m || (!out && cap) || cap < 0) return EWAL_E_INVAL;
  if (!m->valid || m->res.status != EWAL_OK) return 0;
  if (int rc = build_unrec(m)) return rc;
  const int64_t n = std::min<int64_t>(cap, (int64_t)m->unrec.size());
  if (n > 0) std::memcpy(out, m->unrec.data(), (size_t)n * sizeof(ewal_unrec));
  return (int64_t)m->unrec.size();
}

extern "C" int64_t ewal_multi_copy_unrec_bytes(ewal_multi *m, uint8_t *out, int64_t cap) {
  if (!m || (!out && cap) || cap < 0) return EWAL_E_INVAL;
  if (!m->valid || m->res.status != EWAL_OK) return 0;
  if (int rc = build_unrec(m)) return rc;
  const int64_t n = std::min<int64_t>(cap, (int64_t)m->unrec_bytes.size());
  if (n > 0) std::memcpy(out, m->unrec_bytes.data(), (size_t)n);
  return (int64_t)m->unrec_bytes.size();
}

extern "C" int ewal_readall_multi(ewal_ctx *const *ctxs, uint32_t n_ctx, const void *h_buf, uint64_t len,
                                  const uint64_t *file_off, const uint64_t *file_index, uint32_t n_files, uint64_t ri,
                                  ewal_split_result *out, uint32_t *n_resplit) {
  ewal_multi *m = nullptr;
  if (int rc = ewal_multi_create(ctxs, n_ctx, &m)) return rc;
  const int rc = ewal_multi_readall(m, h_buf, len, file_off, file_index, n_files, ri, out);
  if (n_resplit) *n_resplit = m->resplits;
  ewal_multi_destroy(m);
  return rc;
}
