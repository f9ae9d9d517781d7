"""Batched raft.maybeCommit (raft/raft.go:248-258, q() :275-277) followed by
raftLog.maybeCommit / term / at (raft/log.go:115-154, 194-217) over many
independent raft groups, one GPU lane per group (ecommit_batch_device).

Inputs are device buffers (DeviceBuffer) in the SoA layout include/ewal.h
documents: match[v * G + g], nvoters[g] (u8, 1..255), term[g],
committed[g] (updated in place), log_offset[g], log_ptr[G + 1], log_terms.
"""
import ctypes as C

from ._lib import lib, check


def maybe_commit_batch(ctx, G, match, nvoters, term, committed, log_offset, log_ptr, log_terms, changed, status):
    """Returns the device time in ms; changed[g] = maybeCommit's bool,
    status[g] = 0 or EWAL_PANIC_BOUNDS where Go panics."""
    ms = C.c_double()
    check(lib.ecommit_batch_device(ctx.handle, G, match.ptr, nvoters.ptr, term.ptr, committed.ptr, log_offset.ptr,
                                   log_ptr.ptr, log_terms.ptr, changed.ptr, status.ptr, C.byref(ms)))
    return ms.value
