/* ewal_synth.h -- bench / test plumbing: the synthetic WAL generator
 * (etcd_amd/libewal_synth.so, built from etcd_amd/csrc/ewal_synth.cpp).  Not
 * part of the product ABI (include/ewal.h); nothing in libewal.so calls it. */
#pragma once
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Synthetic WAL generator used by bench.py (BASELINE.json configs):
 * Create(metadata) + Save(HardState{1,1,0}, ents) with entry Data sizes
 * log-uniform in [min_data, max_data], payload bytes from xorshift64*(seed),
 * until at least target_bytes.  Writes into out (cap bytes).  Optionally
 * flips one payload byte of record ordinal corrupt_record (-1 = none).
 * Returns bytes written; *n_records receives the frame count. */
int64_t ewal_synth_wal(uint64_t seed, uint64_t target_bytes, uint32_t min_data, uint32_t max_data,
                       int64_t corrupt_record, uint8_t *out, uint64_t cap, int64_t *n_records);
/* The same with rewind_per_mille / 1000 of the entries opening a new
 * leader's term that rewrites the last 1..8 indexes (leader changes);
 * *last_index (nullable) = the last entry's Index. */
int64_t ewal_synth_wal_ex(uint64_t seed, uint64_t target_bytes, uint32_t min_data, uint32_t max_data,
                          int64_t corrupt_record, uint32_t rewind_per_mille, uint8_t *out, uint64_t cap,
                          int64_t *n_records, uint64_t *last_index);

#ifdef __cplusplus
}
#endif
