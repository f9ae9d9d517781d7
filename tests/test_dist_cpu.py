"""Multi-rank combination of shard verdicts (etcd_amd/shard.py) over gloo,
world_size 2 and 4, on CPU: the same code bench.py runs over RCCL."""
import os
import socket
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from etcd_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for c in cases:
            fr, n, failed = c["shards"][rank]
            out.append(shard.combine(dist, rank, fr, n, failed))
        for c in cases:   # commit-index summaries (bench.py --workload commit)
            if "commit" in c:
                ch, lo, hi = c["commit"][rank]
                out.append(tuple(int(x) for x in shard.combine_commit(dist, torch.tensor(ch), torch.tensor(lo),
                                                                       torch.tensor(hi)).tolist()))
        for c in cases:   # the same shards as one batch per rank (bench.py --workload shards)
            if "batch" in c:
                out.append(shard.combine_batch(dist, c["batch_first"][rank], c["batch"][rank]))
        seams = []
        for s in c_seams(cases):
            first, last = s[rank]
            seams.append(shard.seam_check(dist, world, rank, first, last))
        q.put((rank, out, seams))
    finally:
        dist.destroy_process_group()


def c_seams(cases):
    return cases[0].get("seams", [])


def _run(world, cases):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


def test_combine_two_ranks():
    cases = [
        {"shards": [(-1, 1000, False), (-1, 2000, False)],
         "seams": [[(0, 0x1234), (0x1234, 0x99)], [(0, 0x1234), (0x4321, 0x99)], [(0, 0), (0x77, 5)]]},
        {"shards": [(-1, 1000, False), (17, 17, True)]},
        {"shards": [(40, 40, True), (17, 17, True)]},
    ]
    res = _run(2, cases)
    for rank, out, seams in res:
        assert out[0] == (shard.NO_FAILURE, 3000, 0)
        assert shard.decode_key(out[1][0]) == (1, 17) and out[1][1:] == (1017, 1)
        assert shard.decode_key(out[2][0]) == (0, 40) and out[2][1:] == (57, 2)
        # seam: file 1's crc record matches file 0's running CRC / mismatches /
        # running CRC 0 skips the check (wal/wal.go:188)
        assert seams == [-1, 1, -1]


@pytest.mark.timeout(240)
def test_combine_four_ranks():
    cases = [{"shards": [(-1, 10, False), (-1, 20, False), (3, 3, True), (1, 1, True)],
              "seams": [[(0, 5), (5, 6), (6, 7), (7, 8)], [(0, 5), (5, 6), (9, 7), (7, 8)]]}]
    res = _run(4, cases)
    for rank, out, seams in res:
        key, frames, fails = out[0]
        assert shard.decode_key(key) == (2, 3)
        assert frames == 10 + 20 + 3 + 1 and fails == 2
        assert seams == [-1, 2]


def test_combine_batch_two_ranks():
    # rank 0 holds shards 0..2, rank 1 shards 3..5; shard 4 fails at frame 9, shard 1 at frame 30
    cases = [{"shards": [(-1, 1, False), (-1, 1, False)],
              "batch_first": [0, 3],
              "batch": [[(-1, 100, False), (30, 30, True), (-1, 50, False)],
                        [(-1, 10, False), (9, 9, True), (-1, 0, False)]]}]
    res = _run(2, cases)
    for rank, out, seams in res:
        key, frames, fails = out[1]
        assert shard.decode_key(key) == (1, 30)
        assert frames == 100 + 30 + 50 + 10 + 9 and fails == 2


def test_combine_commit_two_ranks():
    cases = [{"shards": [(-1, 1, False), (-1, 1, False)], "commit": [(5, 100, 900), (7, 40, 1200)]}]
    res = _run(2, cases)
    for rank, out, seams in res:
        ch, negmin, hi = out[1]
        assert (ch, -negmin, hi) == (12, 40, 1200)
