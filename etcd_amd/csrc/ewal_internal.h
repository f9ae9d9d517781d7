// ewal_internal.h -- structures shared between the kernels and the host driver.
#pragma once
#include <cstdint>
#include "../../include/ewal.h"

struct TileDesc;

struct Small;
struct StreamArgs {
  const uint8_t *buf;      // WAL bytes (device, 16-B aligned)
  uint64_t B;              // byte count
  uint32_t nunits;         // B / 4096 + 1 (P is read at x == B)
  int find_cand;           // 1: WAL framing candidates, 0: CRC prefixes only
  int ablate;              // unused by k_stream (EWAL_STREAM_ABLATE timing hooks live in k_frame only)
  const uint32_t *g_slice; // [4][256]
  const uint32_t *g_shift; // [48][4][256]
  uint32_t *v;             // lin of every 64-B piece        [nunits*64]
  uint32_t *wcnt;          // candidates in the unit         [nunits]
  uint16_t *slots;         // first EW_SLOTS candidate offsets per unit
  unsigned long long *hmask;   // EW_SPLIT_CAND: per unit, the lanes (64-B pieces) the candidate filter flagged
  Small *small;            // the call's device scratch, zeroed by k_stream's workgroup 0 (of the launch
                           // that starts at unit 0)
  uint32_t u_begin, u_end; // the units this launch covers (a chunk of the stream: u_begin even; all: 0, nunits)
  uint32_t *vh;            // record-dense WALs (the frame pass's 128-B prefixes): the lin of every super-piece's
                           // first 128-B half [nunits*16], else null
  uint32_t *ulin;          // find_cand (EW_ULIN): the lin of every 4 KiB unit [nunits] (the frame pass's phase A)
  const uint32_t *g_unib;  // [16][8][16] nibble tables of S_{256 (15 - m)} for it
};

struct ScanArgs {
  uint32_t nunits, ntiles;        // ntiles = ceil(nunits / EW_TILE_UNITS) (1 MiB tiles)
  const uint32_t *v, *wcnt;       // super-piece lins, candidate counts (k_stream)
  const uint32_t *g_shift;
  uint32_t *ux;                   // lin of every 4 KiB unit          [nunits]
  uint32_t *tagg, *tcnt;          // tile aggregates                  [ntiles]
  uint32_t *tpx;                  // P at every tile start            [ntiles]
  uint32_t *gagg;                 // tile-group (1024 tiles) aggregates [ngroups]
  unsigned long long *gcnt;       // candidates per tile group        [ngroups]
  unsigned long long *tcb;        // candidates before every tile     [ntiles]
  uint32_t *pwave;                // stream prefix at every unit start
  unsigned long long *cbase;      // candidates before every unit
  unsigned long long *total;      // all candidates
  // compaction (find_cand only): slots -> dense sorted candidate list
  const uint16_t *slots;          // nullptr: no compaction
  uint64_t *cpos;
  uint64_t ccap;
  uint32_t *ovf, *novf;           // units with more than EW_SLOTS candidates (k_rescan)
};

// Per-frame descriptor (device), 96 B.
struct RecDesc {
  uint64_t off;            // frame start
  uint64_t doff, dlen;     // Record.Data
  int64_t type;            // Record.Type
  uint32_t crc;            // Record.Crc (stored)
  uint32_t chained;        // decoder CRC after this frame
  int32_t st;              // EWAL_* status of this frame
  int32_t sub_st;          // Entry/HardState Unmarshal status
  uint64_t f0, f1, f2;     // Entry: Term, Index; HardState: Term, Vote, Commit
  uint64_t edoff, edlen;   // Entry.Data
  int32_t etype;           // Entry.Type
  uint8_t dnil, enil;
  uint8_t pad0;            // Record.Data in several segments: 1 not decoded (no room in the side arena),
                           // 2 decoded from their concatenation in the side arena (rd_cat_off)
  uint8_t pad1;            // bit 0: the Entry / HardState carries XXX_unrecognized;
                           // bit 1: Entry.Data lives in the side arena at edoff (a concatenation)
};
// Where the side arena holds a split Record.Data (pad0 == 2): entries keep
// it in f2 (unused by Entry), metadata / HardState frames in edoff.
__host__ __device__ inline uint64_t rd_cat_off(const RecDesc &d) { return d.type == 2 ? d.f2 : d.edoff; }

struct ChainInfo {
  uint32_t last_cand;      // candidate index of the chain's last frame
  uint32_t pad;
};

struct ReadAllAgg {
  unsigned long long first_fail;  // min ordinal with st != 0
  long long last_entry;           // max ordinal of an entry frame
  long long last_state;           // max ordinal of a state frame
  unsigned long long first_meta;  // min ordinal of a non-empty metadata frame
};

// Batched ReadAll over concatenated shards (ewal_readall_batch_device): the
// per-shard reductions of k_check<true>, frame ordinals in the batch.
struct ShardAgg {
  unsigned long long first_fail;  // min frame with st != 0 (~0: none)
  long long last_entry;           // max entry frame (-1)
  long long last_state;           // max state frame (-1)
  unsigned long long first_meta;  // min non-empty metadata frame (~0)
  unsigned long long ent_first;   // global op index of the shard's first entry op (~0)
  uint32_t lastop;                // 1 + the shard's last entry-op frame (0: none)
  uint32_t bad;                   // fused pass: the shard is not on the regular path (replayed alone)
  // fused pass: the shard's frame chain ends before the shard does (a torn
  // tail after a crash, decoder.decode's terminal, wal/decoder.go:30-36)
  uint32_t term1;                 // 1 + the batch frame that ends the shard's frames (0: none)
  int32_t term_st;                // the terminal's class: EWAL_OK (clean io.EOF) or its error
  uint64_t term_off;              // where it sits in the batch
};
// ewal_result.flags bit of a batched shard the fused pass could not decide
// (internal: the host replays the shard alone and clears it)
#define EW_SHARD_BAD 0x40000000
// ... of a batched shard whose entry indexes go back (leader changes): the
// frame pass runs again over its tiles in rewind mode
#define EW_SHARD_REW 0x20000000
// ... whose index rewinds the batch's own frame pass already resolved (the
// shard ran in rewind mode: a ctx's previous batch saw it rewind; round 6)
#define EW_SHARD_REWIN 0x10000000

struct SegArgs {
  uint2 *ulist;            // (frame, op index) of entry ops with XXX_unrecognized (both modes)
  const uint32_t *fs;      // first frame of every shard [ns + 1], fs[ns] = n
  uint32_t ns;
  const uint64_t *ri;      // w.ri of every shard [ns]
  const uint64_t *soff;    // byte offset of every shard in the batch [ns + 1]
  ShardAgg *sagg;          // [ns]
};

// Snapshot verify per-file descriptor.
struct SnapDesc {
  uint64_t off, len;       // file within the packed buffer
  uint64_t doff, dlen;     // snappb.Snapshot.Data
  uint32_t stored, computed;
  int32_t st;
  int32_t resid;           // 1: raftpb.Snapshot needs k_snap_resid, 2: envelope Data split (gather first)
};

// The frame pass's single-WAL verdict words (k_frames / k_frames_seam).  Zero
// means none, so k_stream's zeroing of Small initialises them.
struct FcAgg {
  unsigned long long fail_inv;    // ~((frame << 8) | status) of the first failing frame (max)
  unsigned long long meta_inv;    // ~frame of the first non-empty metadata frame (max)
  uint32_t last_entry1;           // 1 + the last entry frame (max)
  uint32_t last_state1;           // 1 + the last state frame (max)
  uint32_t rare;                  // what the frame pass leaves to the general path or a rerun (frame_kernels.hip:
                                  // 1 declined encoding, 2 index rewind, 4 ents capacity, 8 metadata list, 16 / 32
                                  // far records, 64 rewind slot list, 128 a whole frame after the chain's end)
  uint32_t last_chained;          // the running CRC after the last frame
};

// The frame pass's reductions (k_frames_seam, single WAL): stream positions.
struct FrAgg {
  unsigned long long le, ls;      // 1 + the last entry / state frame's position (max), 0: none
  unsigned long long lo;          // 1 + the last entry op's position (max), 0: none
  unsigned long long nops;        // entry ops
};

// Per-call device scratch (zeroed / initialised each call).
#define EW_ERR_LOOKBACK 1u   // Small.errflag: k_check's look-back gave up waiting (EWAL_E_TIMEOUT)
#define EW_ERR_LIST 2u       // Small.errflag: k_decode met a frame-list index past its capacity (EWAL_E_INVAL)
struct Small {
  uint32_t ticket;
  uint32_t errflag;
  uint32_t novf;
  uint32_t irregular;             // k_link: the candidates do not form one chain from byte 0
  unsigned long long total;       // candidates (k_uscan)
  uint64_t pos0;                  // first candidate position (~0: none)
  uint64_t q;                     // regular chain: offset after the last frame
  int64_t qlen;                   // the int64 at q when q + 8 <= B
  ChainInfo ci;
  ReadAllAgg agg;
  uint32_t nsel;                  // hipcub select counts
  uint32_t nsel2;
  uint32_t nsel3;                 // entry ops
  uint32_t nonmono;               // k_gap: entry indexes not strictly increasing
  uint32_t nmeta;                 // metadata frames listed by k_check
  uint32_t nslow;                 // frames k_decode left to k_decode_slow (non-canonical encodings)
  uint32_t lastop;                // k_check: 1 + the last entry op's frame (0: none)
  uint32_t gapslow;               // k_check: an op's predecessor lies too far back (list-based k_gap)
  uint32_t segbad;                // k_shard_start: a shard does not start on a frame of the chain
  uint32_t spec_n;                // k_spec_gate: frames when k_frame's speculation holds, else 0
  uint32_t nunrec;                // k_check: entry ops carrying XXX_unrecognized (listed in ulist)
  uint32_t fc_done;               // k_frames_seam workgroups done (the last one gathers the result)
  FcAgg fc;
  // the side arena of split byte fields (Go's append over repeated
  // Record.Data / Entry.Data segments, record.pb.go:112, raft.pb.go:254)
  unsigned long long cat_used;    // bytes handed out
  unsigned long long cat_need;    // bytes a frame wanted past the arena's capacity
  uint32_t ncatfail;              // frames left undecoded for want of room (the host grows the arena, reruns)
  uint32_t defer_first;           // a range of a WAL split inside a file (ewal_readall_range_device): frame
                                  // 0's CRC check is the caller's (the running CRC before it is not known here)
  uint32_t fr_capfail;            // batch: the shards' ents regions exceed the capacity (k_shard_rbase)
  FrAgg fr;
  unsigned long long fr_need;     // single WAL: ents the frame pass needed; batch: the regions' total
  uint32_t fr_ncl;                // rewind mode: ents slots claimed more than once (listed for k_ents_fix)
  uint32_t fr_tick;               // k_frames: tiles handed out past the first round (dynamic schedule)
  uint32_t fr_rews;               // single WAL in rewind mode: an index rewind was met (the next call starts so)
  uint32_t fr_below;              // single WAL: an entry with Index < ri was met (not an op)
};

// A returned Entry (ent = its index in ents) or the HardState (ent = -1)
// whose XXX_unrecognized bytes k_unrec gathers into the side buffer.
struct UnrecItem {
  uint32_t r;              // its frame
  uint32_t pad;
  int64_t ent;
  uint64_t off, len;       // in the side buffer
};

// Everything the host needs after the frame pass, gathered by k_result.
struct ResultDev {
  ReadAllAgg agg;
  RecDesc fail, lastent, last, md, sd;
  uint32_t nops, nonmono;
  uint64_t klast;
  uint32_t nslow, gapslow;
  uint32_t errflag, nunrec;
  unsigned long long cat_used, cat_need;
  uint32_t ncatfail, pad;
};
