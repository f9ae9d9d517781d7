"""A longer GPU fuzz run than the suite's (run ON the GPU box): the suite's
tile-spanning large-WAL case (tests/test_gpu_fuzz.py::_large_case) over the
seeds [first, first + count), every result against the oracle, one ctx for all
(stale per-call state shows up as a mismatch); with --batch the batched case
(_large_batch_case, 3-8 such shards per batch); with --split the single case
split inside its file over 2 and 3 ctxs (ewal_readall_multi, the C join).
--repeat (with --batch): every batch twice in a row and then with its shards
in reverse order (the same shard count and bytes): the second call runs the
shards the first saw rewind in rewind mode inside the batch's own pass (the
ctx's hint), the reversed one with a stale hint (round 6).  --vh: the 128-B
prefixes forced on.
Prints one line per 20 seeds.
Usage: python3 tools/fuzz_long.py FIRST COUNT [--batch [--repeat] | --split] [--vh]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from etcd_amd import wal as W          # noqa: E402
from test_gpu_fuzz import _large_batch_case, _large_case, check_batch  # noqa: E402
from test_gpu_multi import _check_full  # noqa: E402
from test_gpu_parity import assert_parity  # noqa: E402


def main():
    first, count = int(sys.argv[1]), int(sys.argv[2])
    ctx = W.Context()
    t0 = time.time()
    statuses = {}
    batch = "--batch" in sys.argv[3:]
    repeat = "--repeat" in sys.argv[3:]
    if "--vh" in sys.argv[3:]:
        ctx.set_options(vh=True)
    split = [W.Context(0) for _ in range(3)] if "--split" in sys.argv[3:] else None
    for s in range(first, first + count):
        if batch:
            shards, ris = _large_batch_case(s)
            got = [r.status for r in check_batch(ctx, shards, ris)]
            if repeat:
                got += [r.status for r in check_batch(ctx, shards, ris)]
                got += [r.status for r in check_batch(ctx, shards[::-1], ris[::-1])]
        elif split:
            m, ri = _large_case(s)
            got = []
            for n in (2, 3):
                g, _ = W.readall_multi(split[:n], m, ri)
                _check_full(m, ri, g, (s, n))
                got.append(g.status)
        else:
            m, ri = _large_case(s)
            got = [assert_parity(ctx, m, ri, check_chain=s % 4 == 0)[0]["status"]]
        for st in got:
            statuses[st] = statuses.get(st, 0) + 1
        if (s - first + 1) % 20 == 0:
            print("seeds %d..%d ok, %.0f s, statuses %s" % (first, s, time.time() - t0, sorted(statuses.items())),
                  flush=True)
    print("done: %d seeds, statuses %s" % (count, sorted(statuses.items())), flush=True)


if __name__ == "__main__":
    main()
