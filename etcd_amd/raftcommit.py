"""Host-side packing for the batched raft.maybeCommit record API
(ecommit_batch_rec_device, include/ewal.h): one 192-B ecommit_group per raft
group -- up to 7 voters' Progress.Match, raftLog.committed, raft.Term, the
log bounds and the terms of the log's last 13 entries (raft/raft.go:248-258,
raft/log.go:115-154) -- built from the SoA arrays ecommit_batch_device takes."""
import numpy as np

RECORD_WORDS = 24   # 192 B
TAIL = 13


def pack_groups(match, nvoters, committed, term, log_offset, log_ptr, log_terms):
    """match: (V, G) uint64 (V >= 1; voters past nvoters[g] are ignored),
    nvoters: (G,) uint8, committed / term / log_offset: (G,) uint64,
    log_ptr: (G + 1,) uint64, log_terms: uint64.  Returns a (G, 24) uint64
    array whose rows are ecommit_group records."""
    match = np.asarray(match, dtype=np.uint64)
    G = match.shape[1]
    nvoters = np.asarray(nvoters)
    # every voter's Match present; a group of more than 7 voters keeps its count in the
    # record (the device reports EWAL_UNSUPPORTED_ENCODING for it: ecommit_batch_device takes those)
    assert int(nvoters.max(initial=0)) <= match.shape[0], "every voter's Match must be present in match"
    rec = np.zeros((G, RECORD_WORDS), dtype=np.uint64)
    nv = min(7, match.shape[0])
    rec[:, :nv] = match[:nv].T
    rec[:, 7] = committed
    rec[:, 8] = term
    rec[:, 9] = log_offset
    lp = np.asarray(log_ptr, dtype=np.uint64)
    nlog = (lp[1:] - lp[:-1]).astype(np.uint64)
    assert int(nlog.max(initial=0)) < 1 << 32, "nlog shares word 10 with nvoters: it must fit 32 bits"
    rec[:, 10] = nlog | (np.asarray(nvoters, dtype=np.uint64) << np.uint64(32))
    lt = np.asarray(log_terms, dtype=np.uint64)
    for k in range(TAIL):
        have = nlog > np.uint64(k)
        idx = (lp[1:] - np.uint64(1) - np.uint64(k))[have].astype(np.int64)
        rec[have, 11 + k] = lt[idx]
    return rec
