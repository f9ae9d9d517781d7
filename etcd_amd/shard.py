"""Multi-GPU combination of per-shard ReadAll results.

WAL replay shards with no data-path exchange: per-raft-group WAL directories
are independent, and inside one WAL every file starts with a crcType record
holding the running CRC at the cut (wal/wal.go:93, 232-234), so files verify
independently.  What crosses ranks is small:

* `combine`   -- one all-reduce of {MIN first-corrupt key, SUM frames, SUM
  failing shards}; key = shard << 40 | frame, so the minimum names the first
  corrupt record of the lowest failing shard.
* `split_verdict` -- ONE WAL split across ranks by file: ReadAll's verdict
  (first failure, its global frame ordinal) from the per-range results,
  with the crc seam and metadata rules across ranges (one all-gather).
* `seam_check` -- for ONE WAL whose files were verified on different ranks:
  the only cross-file rule of ReadAll (wal/wal.go:184-192): file k+1's leading
  crcType record must carry file k's final running CRC whenever that CRC is
  non-zero (otherwise wal.ErrCRCMismatch).  One all-gather of two words per
  rank.

Backend-agnostic (torch.distributed: "nccl" = RCCL on the GPU box, "gloo" in
the CPU tests); tensors live on `device`.
"""
import torch

NO_FAILURE = 1 << 62


def failure_key(shard: int, fail_record: int) -> int:
    """shard << 40 | frame for a failing shard, NO_FAILURE otherwise."""
    return (shard << 40) | fail_record if fail_record >= 0 else NO_FAILURE


def combine(dist, shard: int, fail_record: int, n_records: int, failed: bool, device="cpu", out=None):
    """All-reduce one shard's verdict.  Returns (min key, total frames
    verified, failing shards); frames of a failing shard count up to its first
    failure, as ReadAll's n_records does."""
    t = out if out is not None else torch.zeros(3, dtype=torch.int64, device=device)
    t[0] = failure_key(shard, fail_record)
    t[1] = fail_record if fail_record >= 0 else n_records
    t[2] = 1 if failed else 0
    dist.all_reduce(t[0:1], op=dist.ReduceOp.MIN)
    dist.all_reduce(t[1:3], op=dist.ReduceOp.SUM)
    return int(t[0].item()), int(t[1].item()), int(t[2].item())


def combine_batch(dist, first_shard: int, verdicts, device="cpu", out=None):
    """All-reduce the verdicts of a rank's batch of shards (one batched
    ReadAll, ewal_readall_batch_device): verdicts[i] = (fail_record,
    n_records, failed) of shard first_shard + i.  Same reduction as
    `combine` -- MIN of the failing shards' keys, SUM of frames verified, SUM
    of failing shards -- over the whole batch, in the same one exchange."""
    key, frames, nfail = NO_FAILURE, 0, 0
    for i, (fr, n, failed) in enumerate(verdicts):
        if failed:
            key = min(key, failure_key(first_shard + i, fr))
            nfail += 1
        frames += fr if fr >= 0 else n
    t = out if out is not None else torch.zeros(3, dtype=torch.int64, device=device)
    t[0] = key
    t[1] = frames
    t[2] = nfail
    dist.all_reduce(t[0:1], op=dist.ReduceOp.MIN)
    dist.all_reduce(t[1:3], op=dist.ReduceOp.SUM)
    return int(t[0].item()), int(t[1].item()), int(t[2].item())


def combine_commit(dist, changed, commit_min, commit_max, out=None, device="cpu"):
    """The commit-index summary of a rank's raft-group range after a batched
    maybeCommit (configs[4]): SUM of groups whose commit advanced, MIN and MAX
    commit index over the node -- three words, two all-reduces.  Tensors may
    be device scalars (no host sync before the exchange)."""
    t = out if out is not None else torch.zeros(3, dtype=torch.int64, device=device)
    t[0] = changed
    t[1] = -commit_min    # MAX of the negation == MIN, so one MAX all-reduce carries both
    t[2] = commit_max
    dist.all_reduce(t[0:1], op=dist.ReduceOp.SUM)
    dist.all_reduce(t[1:3], op=dist.ReduceOp.MAX)
    return t


def decode_key(key: int):
    """(shard, frame) of a combined key, or None when no shard failed."""
    if key >= NO_FAILURE:
        return None
    return key >> 40, key & ((1 << 40) - 1)


def seam_check(dist, world: int, rank: int, first_crc_record: int, last_crc: int, device="cpu"):
    """Rank r verified file r of one WAL (files in sequence order).
    first_crc_record: the Crc of the file's leading crcType record (-1 when
    the file does not start with one); last_crc: decoder.lastCRC() after the
    file.  Returns the index of the first file whose seam fails (wal.go:188:
    running != 0 and stored != running), or -1."""
    mine = torch.tensor([first_crc_record, last_crc], dtype=torch.int64, device=device)
    allv = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allv, mine)
    for k in range(1, world):
        running = int(allv[k - 1][1].item())
        stored = int(allv[k][0].item())
        if stored >= 0 and running != 0 and stored != running:
            return k
    return -1


# ---- one WAL split across ranks by file -------------------------------------
# Status numbers of the verdict (include/ewal.h)
_OK, _UNEXPECTED_EOF, _WAL_CRC, _META_CONFLICT, _INDEX_NOT_FOUND = 0, 2, 4, 5, 6
NIL = -2        # a metadata record whose Data is nil
NONE = -1       # no metadata record in the range


def split_verdict(dist, world: int, rank: int, status: int, fail_record: int, n_records: int, last_crc: int,
                  first_crc_record: int, md_first: int, md_first_frame: int, md_last: int, device="cpu"):
    """ReadAll's verdict for ONE WAL whose files were split into contiguous
    ranges, range r verified by rank r (each range starts at a file boundary:
    a crcType record carrying the running CRC, wal/wal.go:93,232-234).  Every
    rank passes its own ReadAll result over its range (with w.ri = the first
    entry index of its range, from the first file's name) plus:
    first_crc_record (the Crc of the range's leading crcType record, -1 if it
    does not start with one), md_first / md_first_frame (a digest of the
    range's first metadata record's Data, NIL for nil Data, NONE when the
    range has none; its frame ordinal in the range) and md_last (the digest
    of the metadata value after the range, as ReadAll returns it).

    One all-gather of 8 words per rank; every rank then walks the ranges in
    file order applying ReadAll's two cross-file rules -- the crc seam
    (wal/wal.go:184-192: running != 0 and stored != running ->
    wal.ErrCRCMismatch) and the metadata rule (wal/wal.go:178-183: metadata !=
    nil and not DeepEqual -> ErrMetadataConflict) -- before each range's own
    first failure.  Returns (status, global frame ordinal of the first
    failure or -1, frames verified, resplit); a range's ErrIndexNotFound (no
    entry at or after its first file's index) is not a failure of the split
    verify.  resplit = k >= 0 when range k (not the last) ends in a torn frame
    (io.ErrUnexpectedEOF at its end): the reference reads on across the file
    boundary (MultiReadCloser), so that frame's verdict depends on the next
    range's bytes -- the caller verifies ranges k.. joined as one range and
    calls again (status is then not final)."""
    mine = torch.tensor([status, fail_record, n_records, last_crc, first_crc_record, md_first, md_first_frame,
                         md_last], dtype=torch.int64, device=device)
    allv = [torch.zeros(8, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allv, mine)
    rows = [[int(x) for x in v.tolist()] for v in allv]
    before, running, md = 0, 0, NONE
    for k, (st, fr, n, lc, fc, mf, mff, ml) in enumerate(rows):
        own = fr if st not in (_OK, _INDEX_NOT_FOUND) else None
        if k > 0 and fc >= 0 and running != 0 and fc != running:
            return _WAL_CRC, before, before, -1
        if k > 0 and md not in (NONE, NIL) and mf != NONE and mf != md and (own is None or mff < own):
            return _META_CONFLICT, before + mff, before + mff, -1
        if own is not None:
            if st == _UNEXPECTED_EOF and k < world - 1 and fr == n:
                return st, before + own, before + own, k
            return st, before + own, before + own, -1
        before += n
        running = lc
        if ml != NONE:
            md = ml
    return _OK, -1, before, -1
