// ewal_host.cpp -- host-side C++ of the engine: wal.OpenAtIndex file
// selection, the write path (encoder/Create/Cut/Save), Snapshotter.Load
// ordering and the host CRC helpers.
//
// None of this decodes or verifies WAL records: ReadAll/loadSnap
// verification runs on the GPU (ewal_api.hip).  The write path computes the
// chained CRC the way wal/encoder.go:25-37 does (crc.Write(Data) then
// rec.Crc = Sum32), with the SSE4.2 crc32 instruction like Go's amd64 path.
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <nmmintrin.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ewal.h"
#include "crc_math.h"
#include "ewal_stage.h"
#include "ewal_wire.h"

namespace {

const uint32_t kCastagnoli = 0x82F63B78u;

std::mutex g_tab_mu;
std::map<uint32_t, std::unique_ptr<ewal::CrcTables>> g_tabs;

const ewal::CrcTables &tables(uint32_t poly) {
  std::lock_guard<std::mutex> lk(g_tab_mu);
  auto it = g_tabs.find(poly);
  if (it != g_tabs.end()) return *it->second;
  auto t = std::make_unique<ewal::CrcTables>(poly);
  const ewal::CrcTables &r = *t;
  g_tabs[poly] = std::move(t);
  return r;
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t crc, const uint8_t *p, size_t n) {
  uint64_t c = (uint32_t)~crc;
  while (n && ((uintptr_t)p & 7)) { c = _mm_crc32_u8((uint32_t)c, *p++); n--; }
  // three independent streams hide the instruction latency on long buffers
  while (n >= 3 * 4096) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t *p1 = p + 4096, *p2 = p + 8192;
    for (int i = 0; i < 4096; i += 8) {
      uint64_t a, b, d;
      std::memcpy(&a, p + i, 8);
      std::memcpy(&b, p1 + i, 8);
      std::memcpy(&d, p2 + i, 8);
      c = _mm_crc32_u64(c, a);
      c1 = _mm_crc32_u64(c1, b);
      c2 = _mm_crc32_u64(c2, d);
    }
    // raw(c, A||B||C) = S_8192(c) ^ S_4096(lin B) ^ lin C  (registers, no inversion)
    static const ewal::CrcTables &t = tables(kCastagnoli);
    c = t.shift_pow2(13, (uint32_t)c) ^ t.shift_pow2(12, (uint32_t)c1) ^ (uint32_t)c2;
    p += 3 * 4096;
    n -= 3 * 4096;
  }
  while (n >= 8) { uint64_t v; std::memcpy(&v, p, 8); c = _mm_crc32_u64(c, v); p += 8; n -= 8; }
  while (n) { c = _mm_crc32_u8((uint32_t)c, *p++); n--; }
  return ~(uint32_t)c;
}

uint32_t crc_update(uint32_t crc, uint32_t poly, const uint8_t *p, size_t n) {
  if (poly == kCastagnoli && __builtin_cpu_supports("sse4.2")) return crc32c_hw(crc, p, n);
  return tables(poly).update(crc, p, n);
}

using namespace ewal_wire;

// ---- wal file names, wal/util.go:20-88 -------------------------------------
// fmt.Sscanf(str, "%016x-%016x.wal", &seq, &index): hex fields of at most 16
// digits, literal '-' and ".wal"; trailing text is not examined.
bool scan_hex16(const char *&s, uint64_t &v) {
  v = 0;
  int n = 0;
  while (n < 16) {
    char ch = *s;
    int d;
    if (ch >= '0' && ch <= '9') d = ch - '0';
    else if (ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
    else if (ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
    else break;
    v = (v << 4) | (uint64_t)d;
    ++s;
    ++n;
  }
  return n > 0;
}
bool parse_wal_name(const std::string &name, uint64_t *seq, uint64_t *index) {
  const char *s = name.c_str();
  uint64_t a = 0, b = 0;
  if (!scan_hex16(s, a)) return false;
  if (*s != '-') return false;
  ++s;
  if (!scan_hex16(s, b)) return false;
  if (std::strncmp(s, ".wal", 4) != 0) return false;
  *seq = a;
  *index = b;
  return true;
}
std::string wal_name(uint64_t seq, uint64_t index) {
  char b[64];
  std::snprintf(b, sizeof b, "%016llx-%016llx.wal", (unsigned long long)seq, (unsigned long long)index);
  return b;
}
bool read_dir(const std::string &dir, std::vector<std::string> *names) {
  DIR *d = opendir(dir.c_str());
  if (!d) return false;
  while (dirent *e = readdir(d)) {
    std::string n = e->d_name;
    if (n == "." || n == "..") continue;
    names->push_back(n);
  }
  closedir(d);
  return true;
}
bool read_file(const std::string &path, std::vector<uint8_t> *out, size_t pad) {
  FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  size_t base = out->size();
  out->resize(base + (size_t)sz + pad);
  size_t got = sz ? std::fread(out->data() + base, 1, (size_t)sz, f) : 0;
  std::fclose(f);
  out->resize(base + got);
  return got == (size_t)sz;
}

}  // namespace

// ===========================================================================
// An opened WAL (wal.OpenAtIndex): the selected files names[nameIndex:]; their
// bytes are read (as MultiReadCloser streams them, wal/wal.go:126-134) into
// one host buffer -- the buffer ReadAll's ents are views into -- by a small
// pool of reader threads, in pieces of at most kPiece bytes.  The reading
// starts at ewal_wal_prefetch (or at ReadAll), so it can run while the
// caller creates the GPU context; ReadAll uploads every piece, in order, as
// soon as it and all earlier ones are in the buffer.
namespace {
const uint64_t kPiece = 64ull << 20;
struct Piece {
  size_t file;
  uint64_t foff, off, len;
};
}  // namespace

struct ewal_wal {
  std::string dir;
  uint64_t ri = 0;
  uint64_t seq = 0;
  std::vector<std::string> paths;
  std::vector<uint64_t> sizes;
  uint64_t total = 0;
  uint8_t *bytes = nullptr;           // total bytes once loaded (anonymous mapping, huge pages advised)
  size_t map_len = 0;
  bool loaded = false;
  // the reader pool (started once)
  bool started = false;
  std::vector<Piece> pcs;
  std::vector<int> fds;
  std::unique_ptr<std::atomic<int>[]> done;   // per piece: 0 pending, 1 read, -1 failed
  std::atomic<size_t> next{0};
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> th;
  void stop() {
    next.store(pcs.size());   // no more pieces handed out
    for (auto &t : th) t.join();
    th.clear();
    for (int fd : fds)
      if (fd >= 0) close(fd);
    fds.clear();
  }
  ~ewal_wal() {
    stop();
    if (bytes) munmap(bytes, map_len);
  }
};

namespace {

// Start reading every piece (idempotent): the buffer, the files, the pool.
int start_load(ewal_wal *w) {
  if (w->started || w->loaded) return EWAL_OK;
  uint64_t off = 0;
  for (size_t f = 0; f < w->paths.size(); ++f)
    for (uint64_t o = 0; o < w->sizes[f]; o += kPiece) {
      const uint64_t l = std::min<uint64_t>(kPiece, w->sizes[f] - o);
      w->pcs.push_back(Piece{f, o, off, l});
      off += l;
    }
  if (!w->bytes) {
    // one anonymous mapping in 2 MiB huge pages where the kernel allows:
    // first-touch faults per 4 KiB page otherwise dominate the read
    const size_t hp = 2u << 20;
    w->map_len = (size_t)((std::max<uint64_t>(w->total, 1) + hp - 1) / hp * hp);
    void *m = mmap(nullptr, w->map_len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) {
      w->map_len = 0;
      w->pcs.clear();
      return EWAL_E_NOMEM;
    }
    (void)madvise(m, w->map_len, MADV_HUGEPAGE);
    w->bytes = (uint8_t *)m;
  }
  w->fds.assign(w->paths.size(), -1);
  for (size_t f = 0; f < w->paths.size(); ++f) {
    w->fds[f] = open(w->paths[f].c_str(), O_RDONLY);
    if (w->fds[f] < 0) {
      w->stop();
      w->pcs.clear();
      return EWAL_E_IO;
    }
  }
  w->done.reset(new std::atomic<int>[std::max<size_t>(1, w->pcs.size())]);
  for (size_t k = 0; k < w->pcs.size(); ++k) w->done[k].store(0);
  w->next.store(0);
  auto reader = [w]() {
    for (;;) {
      const size_t k = w->next.fetch_add(1);
      if (k >= w->pcs.size()) break;
      const Piece &p = w->pcs[k];
      uint64_t got = 0;
      while (got < p.len) {
        const ssize_t r = pread(w->fds[p.file], w->bytes + p.off + got, (size_t)(p.len - got), (off_t)(p.foff + got));
        if (r <= 0) break;
        got += (uint64_t)r;
      }
      {
        std::lock_guard<std::mutex> lk(w->mu);
        w->done[k].store(got == p.len ? 1 : -1);
      }
      w->cv.notify_all();
    }
  };
  const unsigned nth = (unsigned)std::max<size_t>(
      1, std::min<size_t>(w->pcs.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency()))));
  for (unsigned t = 0; t < nth; ++t) w->th.emplace_back(reader);
  w->started = true;
  return EWAL_OK;
}

// Every piece, in order, to `ready` as soon as it and all earlier ones are
// in the buffer (ReadAll uploads them while the later ones are still read).
template <class F>
int load_pieces(ewal_wal *w, F ready) {
  if (w->loaded) return w->total ? ready(0, w->total) : EWAL_OK;
  int rc = start_load(w);
  if (rc) return rc;
  for (size_t k = 0; k < w->pcs.size(); ++k) {
    std::unique_lock<std::mutex> lk(w->mu);
    w->cv.wait(lk, [&] { return w->done[k].load() != 0; });
    lk.unlock();
    if (w->done[k].load() < 0) { rc = EWAL_E_IO; break; }
    if ((rc = ready(w->pcs[k].off, w->pcs[k].len)) != 0) break;
  }
  w->stop();
  w->started = false;
  w->pcs.clear();
  if (rc == EWAL_OK) w->loaded = true;
  return rc;
}

}  // namespace

struct ewal_encoder {
  std::vector<uint8_t> buf;
  uint32_t crc = 0;
};

struct ewal_writer {
  std::string dir;
  std::vector<uint8_t> md;
  bool md_nil = true;
  uint64_t seq = 0, enti = 0;
  int fd = -1;
  ewal_encoder enc;
};

extern "C" {

const char *ewal_status_string(int st) {
  switch (st) {
  case EWAL_OK: return "ok";
  case EWAL_EOF: return "EOF";
  case EWAL_ERR_UNEXPECTED_EOF: return "unexpected EOF";
  case EWAL_ERR_RECORD_CRC: return "walpb: crc mismatch";
  case EWAL_ERR_WAL_CRC: return "wal: crc mismatch";
  case EWAL_ERR_METADATA_CONFLICT: return "wal: conflicting metadata found";
  case EWAL_ERR_INDEX_NOT_FOUND: return "wal: index not found in file";
  case EWAL_ERR_WRONG_TYPE: return "proto: field/encoding mismatch: wrong type for field";
  case EWAL_ERR_UNEXPECTED_TYPE: return "unexpected block type";
  case EWAL_ERR_FILE_NOT_FOUND: return "wal: file not found";
  case EWAL_ERR_SNAP_CRC: return "snap: crc mismatch";
  case EWAL_ERR_NO_SNAPSHOT: return "snap: no available snapshot";
  case EWAL_PANIC_NEG_LENGTH: return "panic: makeslice: len out of range";
  case EWAL_PANIC_BOUNDS: return "panic: runtime error: slice bounds out of range";
  case EWAL_PANIC_ENTRY: return "panic: mustUnmarshalEntry";
  case EWAL_PANIC_STATE: return "panic: mustUnmarshalState";
  case EWAL_PANIC_INDEX_GAP: return "panic: ents index gap";
  case EWAL_NONTERMINATING: return "reference does not terminate";
  case EWAL_UNSUPPORTED_ENCODING: return "unsupported (non-canonical) record encoding";
  case EWAL_E_HIP: return "HIP error";
  case EWAL_E_INVAL: return "invalid argument";
  case EWAL_E_NOMEM: return "out of memory";
  case EWAL_E_NODEVICE: return "no GPU device";
  case EWAL_E_TIMEOUT: return "device timeout";
  case EWAL_E_IO: return "I/O error";
  default: return "unknown";
  }
}

uint32_t ewal_crc32_update_host(uint32_t crc, uint32_t poly, const uint8_t *p, uint64_t n) {
  return crc_update(crc, poly, p, (size_t)n);
}

uint32_t ewal_crc32_combine(uint32_t poly, uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return tables(poly).combine(crc_a, crc_b, len_b);
}

// ---- wal file names, wal/util.go:20-88 ---------------------------------------
int ewal_parse_wal_name(const char *name, uint64_t *seq, uint64_t *index) {
  uint64_t a = 0, b = 0;
  if (!name || !parse_wal_name(name, &a, &b)) return 0;
  if (seq) *seq = a;
  if (index) *index = b;
  return 1;
}

int64_t ewal_search_index(const char *const *names, uint64_t n, uint64_t index) {
  for (uint64_t k = n; k-- > 0;) {
    uint64_t s, i;
    if (!parse_wal_name(names[k], &s, &i)) return EWAL_E_INVAL;   // Go: panic("parse correct name error")
    if (index >= i) return (int64_t)k;
  }
  return -1;
}

int ewal_is_valid_seq(const char *const *names, uint64_t n) {
  uint64_t last = 0;
  for (uint64_t k = 0; k < n; ++k) {
    uint64_t s, i;
    if (!parse_wal_name(names[k], &s, &i)) return EWAL_E_INVAL;
    if (last != 0 && last != s - 1) return 0;
    last = s;
  }
  return 1;
}

void ewal_wal_name(uint64_t seq, uint64_t index, char *out) {
  std::snprintf(out, 38, "%016llx-%016llx.wal", (unsigned long long)seq, (unsigned long long)index);
}

// ---- wal.OpenAtIndex, wal/wal.go:108-159 ------------------------------------
int ewal_open_at_index(const char *dirpath, uint64_t index, ewal_wal **out) {
  *out = nullptr;
  std::vector<std::string> all, names;
  if (!read_dir(dirpath, &all)) return EWAL_E_IO;
  for (auto &n : all) {   // checkWalNames
    uint64_t s, i;
    if (parse_wal_name(n, &s, &i)) names.push_back(n);
  }
  if (names.empty()) return EWAL_ERR_FILE_NOT_FOUND;
  std::sort(names.begin(), names.end());
  std::vector<const char *> np;
  for (auto &n : names) np.push_back(n.c_str());
  const int64_t ni = ewal_search_index(np.data(), np.size(), index);
  if (ni < 0) return EWAL_ERR_FILE_NOT_FOUND;
  if (ewal_is_valid_seq(np.data() + ni, np.size() - (size_t)ni) != 1) return EWAL_ERR_FILE_NOT_FOUND;
  auto *w = new ewal_wal();
  w->dir = dirpath;
  w->ri = index;
  for (size_t k = (size_t)ni; k < names.size(); ++k) {   // os.Open of each file (wal/wal.go:126-133)
    const std::string p = std::string(dirpath) + "/" + names[k];
    struct stat st;
    if (stat(p.c_str(), &st) != 0 || access(p.c_str(), R_OK) != 0) {
      delete w;
      return EWAL_E_IO;
    }
    w->paths.push_back(p);
    w->sizes.push_back((uint64_t)st.st_size);
    w->total += (uint64_t)st.st_size;
  }
  uint64_t s, i;
  parse_wal_name(names.back(), &s, &i);
  w->seq = s;
  *out = w;
  return EWAL_OK;
}

uint64_t ewal_wal_size(ewal_wal *w) { return w ? w->total : 0; }

// (*WAL).ReadAll over the opened files: the files are read in 64 MiB pieces
// by a few threads while every finished piece is already on its way to HBM
// (ewal_stage_put, asynchronous on the ctx stream), then the device pipeline
// runs on the staged bytes.
int ewal_wal_readall(ewal_wal *w, ewal_ctx *ctx, ewal_result *out) {
  if (!w || !out) return EWAL_E_INVAL;
  int rc = ewal_stage_begin(ctx, w->total);
  if (rc) return rc;
  rc = load_pieces(w, [&](uint64_t off, uint64_t len) { return ewal_stage_put(ctx, off, w->bytes + off, len); });
  if (rc) {
    // copies already queued read w->bytes: let them land before the caller can
    // unmap it (ewal_wal_close)
    (void)ewal_stage_sync(ctx);
    return rc;
  }
  return ewal_stage_readall(ctx, w->total, w->ri, out);
}

const uint8_t *ewal_wal_bytes(ewal_wal *w, uint64_t *len) {
  if (!w) return nullptr;
  if (!w->loaded && load_pieces(w, [](uint64_t, uint64_t) { return 0; }) != EWAL_OK) {
    if (len) *len = 0;
    return nullptr;
  }
  if (len) *len = w->total;
  return w->bytes;
}
int ewal_wal_prefetch(ewal_wal *w) {
  if (!w) return EWAL_E_INVAL;
  return start_load(w);
}
uint64_t ewal_wal_seq(ewal_wal *w) { return w->seq; }
void ewal_wal_close(ewal_wal *w) { delete w; }

// ---- encoder.encode, wal/encoder.go:25-37 ------------------------------------
ewal_encoder *ewal_encoder_new(uint32_t prev_crc, uint64_t reserve) {
  auto *e = new ewal_encoder();
  e->crc = prev_crc;
  if (reserve) e->buf.reserve((size_t)reserve);
  return e;
}
int ewal_encoder_encode(ewal_encoder *e, int64_t type, const uint8_t *data, uint64_t n, int data_nil) {
  const bool nil = data_nil != 0;
  e->crc = crc_update(e->crc, kCastagnoli, data, nil ? 0 : (size_t)n);
  const size_t sz = frame_size(type, e->crc, n, nil);
  const size_t base = e->buf.size();
  e->buf.resize(base + sz);
  frame_write(e->buf.data() + base, type, e->crc, data, n, nil);
  return EWAL_OK;
}
int ewal_encoder_save_entry(ewal_encoder *e, int32_t type, uint64_t term, uint64_t index, const uint8_t *data,
                            uint64_t n) {
  std::vector<uint8_t> b(entry_size(type, term, index, n));
  entry_marshal(b.data(), type, term, index, data, n);
  return ewal_encoder_encode(e, EWAL_ENTRY, b.data(), b.size(), 0);
}
int ewal_encoder_save_state(ewal_encoder *e, uint64_t term, uint64_t vote, uint64_t commit) {
  if (term == 0 && vote == 0 && commit == 0) return EWAL_OK;   // raft.IsEmptyHardState
  uint8_t b[40];
  size_t n = state_marshal(b, term, vote, commit);
  return ewal_encoder_encode(e, EWAL_STATE, b, n, 0);
}
const uint8_t *ewal_encoder_bytes(ewal_encoder *e, uint64_t *len) {
  if (len) *len = e->buf.size();
  return e->buf.data();
}
uint32_t ewal_encoder_crc(ewal_encoder *e) { return e->crc; }
void ewal_encoder_free(ewal_encoder *e) { delete e; }

// ---- Create / Cut / Save / Sync, wal/wal.go:72-100, 219-292 ------------------
static int writer_flush(ewal_writer *w) {
  const uint8_t *p = w->enc.buf.data();
  size_t n = w->enc.buf.size();
  while (n) {
    ssize_t k = ::write(w->fd, p, n);
    if (k < 0) {
      if (errno == EINTR) continue;
      return EWAL_E_IO;
    }
    p += k;
    n -= (size_t)k;
  }
  w->enc.buf.clear();
  return EWAL_OK;
}
static int writer_open(ewal_writer *w, uint64_t seq, uint64_t index) {
  std::string p = w->dir + "/" + wal_name(seq, index);
  w->fd = ::open(p.c_str(), O_WRONLY | O_APPEND | O_CREAT, 0600);
  return w->fd < 0 ? EWAL_E_IO : EWAL_OK;
}
int ewal_create(const char *dirpath, const uint8_t *md, uint64_t mlen, int md_nil, ewal_writer **out) {
  *out = nullptr;
  std::vector<std::string> names;
  if (read_dir(dirpath, &names) && !names.empty()) { errno = EEXIST; return EWAL_E_IO; }   // os.ErrExist
  std::string cmd = dirpath;
  // os.MkdirAll(dirpath, 0700)
  for (size_t i = 1; i <= cmd.size(); ++i)
    if (i == cmd.size() || cmd[i] == '/') ::mkdir(cmd.substr(0, i).c_str(), 0700);
  auto *w = new ewal_writer();
  w->dir = dirpath;
  w->md.assign(md, md + (md_nil ? 0 : mlen));
  w->md_nil = md_nil != 0;
  if (writer_open(w, 0, 0) != EWAL_OK) { delete w; return EWAL_E_IO; }
  w->enc.crc = 0;
  ewal_encoder_encode(&w->enc, EWAL_CRC, nullptr, 0, 1);        // saveCrc(0)
  ewal_encoder_encode(&w->enc, EWAL_METADATA, w->md.data(), w->md.size(), w->md_nil);
  *out = w;
  return EWAL_OK;
}
int ewal_writer_save_entry(ewal_writer *w, int32_t type, uint64_t term, uint64_t index, const uint8_t *data,
                           uint64_t n) {
  ewal_encoder_save_entry(&w->enc, type, term, index, data, n);
  w->enti = index;
  return EWAL_OK;
}
int ewal_writer_save_state(ewal_writer *w, uint64_t term, uint64_t vote, uint64_t commit) {
  return ewal_encoder_save_state(&w->enc, term, vote, commit);
}
int ewal_writer_sync(ewal_writer *w) {
  int rc = writer_flush(w);
  if (rc) return rc;
  return ::fsync(w->fd) == 0 ? EWAL_OK : EWAL_E_IO;
}
int ewal_writer_cut(ewal_writer *w) {
  // (*WAL).Cut, wal/wal.go:219-238: the next file is opened first; when that
  // fails the WAL keeps writing to the current one.  Then the current file
  // is synced (its error ignored, as w.Sync() is there) and closed, and the
  // new one takes its place.
  const uint64_t nseq = w->seq + 1, nidx = w->enti + 1;
  const std::string np = w->dir + "/" + wal_name(nseq, nidx);
  const int nfd = ::open(np.c_str(), O_WRONLY | O_APPEND | O_CREAT, 0600);
  if (nfd < 0) return EWAL_E_IO;
  (void)ewal_writer_sync(w);   // w.Sync()'s error is not checked in Cut either
  ::close(w->fd);
  w->fd = nfd;
  w->seq = nseq;
  // newEncoder(w.f, prevCrc): a fresh buffer (bytes a failed sync left
  // behind belong to the old file and are dropped), the running CRC kept
  w->enc.buf.clear();
  // saveCrc(prevCrc): Cut returns its error before the metadata record
  // (wal/wal.go:234-236)
  if (int rc = ewal_encoder_encode(&w->enc, EWAL_CRC, nullptr, 0, 1)) return rc;
  return ewal_encoder_encode(&w->enc, EWAL_METADATA, w->md.data(), w->md.size(), w->md_nil);
}
void ewal_writer_close(ewal_writer *w) {
  if (!w) return;
  if (w->fd >= 0) {
    ewal_writer_sync(w);
    ::close(w->fd);
  }
  delete w;
}

// ---- Snapshotter.Load, snap/snapshotter.go:62-74, 76-111, 115-150 ----------
// snapNames: the directory's *.snap names, newest (largest) first
static int snap_names(const char *dirpath, std::vector<std::string> *snaps) {
  std::vector<std::string> all;
  if (!read_dir(dirpath, &all)) return EWAL_E_IO;
  for (auto &n : all)   // checkSuffix
    if (n.size() >= 5 && n.compare(n.size() - 5, 5, ".snap") == 0) snaps->push_back(n);
  if (snaps->empty()) return EWAL_ERR_NO_SNAPSHOT;
  std::sort(snaps->rbegin(), snaps->rend());   // sort.Reverse(sort.StringSlice)
  return EWAL_OK;
}

int64_t esnap_names(const char *dirpath, char *out, uint64_t cap, uint64_t *len) {
  std::vector<std::string> snaps;
  const int st = snap_names(dirpath, &snaps);
  if (st != EWAL_OK) return st == EWAL_ERR_NO_SNAPSHOT ? 0 : st;
  std::string joined;
  for (auto &n : snaps) {
    joined += n;
    joined.push_back('\0');
  }
  if (len) *len = joined.size();
  if (out && cap) std::memcpy(out, joined.data(), std::min<uint64_t>(cap, joined.size()));
  return (int64_t)snaps.size();
}

int esnap_load_dir(ewal_ctx *ctx, const char *dirpath, uint32_t poly, esnap_snapshot *out, char **out_name) {
  if (out_name) *out_name = nullptr;
  std::vector<std::string> snaps;
  const int sn = snap_names(dirpath, &snaps);
  if (sn != EWAL_OK) return sn;
  int err = EWAL_ERR_NO_SNAPSHOT;
  for (auto &name : snaps) {
    const std::string path = std::string(dirpath) + "/" + name;
    std::vector<uint8_t> b;
    int st;
    if (!read_file(path, &b, 0)) {
      st = EWAL_E_IO;
    } else {
      // one-file batch on the GPU
      void *d = nullptr;
      int rc = ewal_stage_to_device(ctx, b.data(), b.size(), &d);
      if (rc) return rc;
      uint64_t off = 0, len = b.size();
      int32_t s = 0;
      rc = esnap_verify_packed(ctx, d, len, &off, &len, 1, poly, &s, nullptr, nullptr);
      if (rc) return rc;
      st = s;
      if (st == EWAL_OK) {
        rc = esnap_copy_snapshot(ctx, 0, out);
        if (rc) return rc;
        if (out_name) *out_name = strdup(name.c_str());
        return EWAL_OK;
      }
    }
    // loadSnap's deferred renameBroken runs only on the errors Go returns
    // (read error, snappb / raftpb Unmarshal errors, ErrCRCMismatch).  A Go
    // panic (bounds, non-termination) propagates out of Load instead, and
    // EWAL_UNSUPPORTED_ENCODING is a limit of this engine (a valid file Go
    // would load): both stop here with the file left in place, so the caller
    // can decode it on the host.
    const bool go_error = st == EWAL_E_IO || st == EWAL_ERR_SNAP_CRC || st == EWAL_ERR_UNEXPECTED_EOF ||
                          st == EWAL_ERR_WRONG_TYPE;
    if (!go_error) {
      if (out_name) *out_name = strdup(name.c_str());
      return st;
    }
    err = st;
    std::string broken = path + ".broken";   // renameBroken
    if (std::rename(path.c_str(), broken.c_str()) != 0)
      std::fprintf(stderr, "Cannot rename broken snapshot file %s to %s\n", path.c_str(), broken.c_str());
  }
  return err;
}

}  // extern "C"
