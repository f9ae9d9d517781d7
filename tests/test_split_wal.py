"""ONE WAL split across ranks by file (each file starts with a
crcType record carrying the running CRC, wal/wal.go:93,232-234): every rank
runs ReadAll over its contiguous range of files, then shard.split_verdict's
one all-gather applies ReadAll's cross-file rules (crc seam, metadata) in file
order.  The global verdict must equal ReadAll over all the files.

CPU (gloo, world_size 2 and 3): each range's result comes from the oracle's
ReadAll of that range.  GPU (-m gpu, world_size 2 on one MI355X, gloo for the
exchange): each range's result comes from the engine (libewal.so)."""
import os
import random
import socket
import struct

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from etcd_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def md_digest(b):
    return shard.NIL if b is None else (len(b) << 32) | O.crc32_update(0, b)


def build_files(rng, nfiles, md=b"metadata", md_override=None, ents=(5, 60)):
    """wal.Create + Save + Cut ... as the reference writes them: file k starts
    with crcType{running CRC} and metadataType{md}; returns [(bytes, first
    entry index)]."""
    files, prev, idx = [], 0, 0
    for k in range(nfiles):
        e = O.WalEncoder(prev)
        e.save_crc(prev)
        e.encode(1, md_override.get(k, md) if md_override else md)
        first = idx
        for _ in range(rng.randrange(*ents)):
            e.save_entry(0, 1, idx, rng.randbytes(rng.randrange(0, 2000)))
            idx += 1
        e.save_state(1, 1, idx)
        files.append((e.getvalue(), first))
        prev = e.crc
    return files


def range_inputs(buf, ri, result):
    """split_verdict's per-rank inputs from a range's ReadAll result and its
    decoded records [(type, crc, data)]."""
    st, fr, n, lc, md = result
    recs, p = [], 0                      # the frames' records (int64 length + Record.Unmarshal), no CRC check
    while p + 8 <= len(buf):
        L = struct.unpack_from("<q", buf, p)[0]
        if L < 0 or p + 8 + L > len(buf):
            break
        rs, r = O.record_unmarshal(buf[p + 8:p + 8 + L])
        if rs != O.OK:
            break
        recs.append((r["type"], r["crc"], r["data"]))
        p += 8 + L
    fc = recs[0][1] if recs and recs[0][0] == 4 else -1
    mi = next((i for i, r in enumerate(recs) if r[0] == 1), None)
    mf, mff = (shard.NONE, -1) if mi is None else (md_digest(recs[mi][2] if recs[mi][2] else None), mi)
    ml = md_digest(md) if any(r[0] == 1 for r in recs[:n if st == O.OK else fr]) else shard.NONE
    return st, fr, n, lc, fc, mf, mff, ml


def oracle_result(buf, ri):
    o = O.readall(buf, ri)
    return o["status"], o["fail_record"], o["n_records"], o["last_crc"], o["metadata"]


def _worker(rank, world, port, cases, use_gpu, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = None
        if use_gpu:
            from etcd_amd import wal as W
            ctx = W.Context(0)
        out = []
        for ranges in cases:
            ranges = list(ranges)
            while True:
                buf, ri = ranges[rank]
                if use_gpu:
                    g = W.readall_bytes(buf, ri, ctx, with_ents=False)
                    res = (g.status, g.fail_record, g.n_records, g.last_crc, g.metadata)
                else:
                    res = oracle_result(buf, ri)
                v = shard.split_verdict(dist, world, rank, *range_inputs(buf, ri, res))
                if v[3] < 0:
                    break
                # a torn frame at the end of range k: ranges k.. verified joined, on rank k
                k = v[3]
                ranges = ranges[:k] + [(b"".join(b for b, _ in ranges[k:]), ranges[k][1])] + \
                    [(b"", 0)] * (world - k - 1)
                out.append(("resplit", k))
            out.append(v[:3])
        if ctx is not None:
            ctx.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _cases(rng, world):
    """[(all bytes, [per-rank (range bytes, ri)])] over clean / corrupt /
    seam / metadata-conflict WALs."""
    out = []
    for kind in ("clean", "corrupt_late", "corrupt_both", "seam", "meta", "meta_nil", "torn"):
        nf = world * 2
        over = {nf // 2: b"other"} if kind == "meta" else ({1: None} if kind == "meta_nil" else None)
        files = build_files(rng, nf, md_override=over)
        blobs = [bytearray(b) for b, _ in files]
        if kind == "corrupt_late":
            blobs[-1][len(blobs[-1]) // 2] ^= 0x10
        if kind == "corrupt_both":
            blobs[0][len(blobs[0]) - 30] ^= 0x10
            blobs[-1][len(blobs[-1]) // 2] ^= 0x10
        if kind == "seam":     # the crcType record of the file opening the last range carries a wrong CRC
            k = nf - 2
            c = O.WalEncoder(12345)
            c.save_crc(12345)
            fixed = c.getvalue()
            old = O.WalEncoder(0)
            old.save_crc(0)
            head = len(old.getvalue())    # 12-byte crc record when the CRC varint is short; rebuild the file
            b2 = O.WalEncoder(12345)
            b2.save_crc(12345)
            body = bytes(blobs[k])[8 + blobs[k][0]:]
            blobs[k] = bytearray(b2.getvalue() + body)
            assert fixed and head
        if kind == "torn":          # the last file of range 0 torn: its frame reads on into range 1
            blobs[nf // world - 1] = blobs[nf // world - 1][:-5]
        per = nf // world
        ranges = []
        for r in range(world):
            part = b"".join(bytes(x) for x in blobs[r * per:(r + 1) * per])
            ranges.append((part, 0 if r == 0 else files[r * per][1]))
        out.append((b"".join(bytes(x) for x in blobs), ranges))
    return out


def _run(world, use_gpu):
    rng = random.Random(17 + world)
    cases = _cases(rng, world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, [c[1] for c in cases], use_gpu, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        got = [x for x in res[r] if x[0] != "resplit"]
        assert len(got) == len(cases)
        assert any(x[0] == "resplit" for x in res[r])       # the torn-file case went through a resplit
        for i, (allb, _) in enumerate(cases):
            o = O.readall(allb, 0)
            want = (o["status"], o["fail_record"] if o["status"] != O.OK else -1)
            st, fr, _ = got[i]
            assert (st, fr) == want, (i, r, (st, fr), want)
    return cases


@pytest.mark.parametrize("world", [2, 3])
def test_split_verdict_oracle_ranges(world):
    cases = _run(world, use_gpu=False)
    kinds = [O.readall(c[0], 0)["status"] for c in cases]
    assert O.ERR_WAL_CRC in kinds and O.ERR_METADATA_CONFLICT in kinds and O.ERR_RECORD_CRC in kinds


@pytest.mark.gpu
def test_split_verdict_gpu_ranges():
    _run(2, use_gpu=True)
