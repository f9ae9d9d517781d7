"""ONE WAL split across ranks INSIDE a file ("within one file,
split at record boundaries"; the cross-rank prefix combination is one
(CRC, length) exchange): rank r starts at the first frame-start candidate
after r * len / world (ewal_range_probe), runs ReadAll over its range with
frame 0's CRC check deferred (ewal_readall_range_device), and
shard.split_verdict makes that check with the running CRC of the ranges
before -- crc32.Update(running, Data0) from (crc32.Update(0, Data0), len) by
ewal_crc32_combine -- while applying ReadAll's other cross-range rules.  The
joined verdict must equal ReadAll over the whole WAL.

CPU (gloo, world 2 and 3): each range's result comes from the oracle run on
the range behind a crcType record carrying the true running CRC (a test-side
stand-in for the deferred check; cases whose frame 0 itself is corrupt are
GPU-only).  GPU (-m gpu): the product alone -- probe, range ReadAll, range
info -- on 2 and 3 ranks sharing the MI355X, gloo for the exchange."""
import datetime
import os
import random
import traceback
import socket
import struct

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from etcd_amd import shard
from test_split_wal import oracle_range_info


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wal(rng, n=300, cuts=2, md=b"metadata", max_data=1500):
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, md)
    idx = 1
    cut_at = set(rng.sample(range(10, n), cuts))
    out = b""
    for i in range(n):
        if i in cut_at:      # wal.Cut: a new file opens with crcType{running CRC} + metadata
            out += e.getvalue()
            prev = e.crc
            e = O.WalEncoder(prev)
            e.save_crc(prev)
            e.encode(1, md)
        if i % 37 == 5:
            e.save_state(1, 1, idx)
        e.save_entry(0, 1, idx, rng.randbytes(rng.randrange(0, max_data)))
        idx += 1
    return out + e.getvalue()


def _frames(buf):
    """frame offsets along the chain from 0 (test helper)"""
    offs, p = [], 0
    while p + 8 <= len(buf):
        L = struct.unpack_from("<q", buf, p)[0]
        if L < 0 or p + 8 + L > len(buf):
            break
        offs.append(p)
        p += 8 + L
    return offs


def _cases(rng):
    """(kind, WAL bytes, global ri, frame-0-corrupt: GPU only)"""
    out = []
    w = _wal(rng)
    out.append(("clean", w, 1, False))
    out.append(("ri_mid", w, 40, False))
    offs = _frames(w)
    b = bytearray(w)                   # a record's Data flipped in the middle of the WAL
    b[offs[len(offs) * 2 // 3] + 30] ^= 0x04
    out.append(("corrupt_mid", bytes(b), 1, False))
    # every entry's Data is a run of false frame-start candidates: a share
    # boundary lands inside one, the range starting there is not on the chain
    # (the range before it ends in a frame cut short) and is verified joined
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"m")
    fake = struct.pack("<q", 40) + bytes([0x08, 0x02, 0x10, 0x05]) + bytes(36)
    for i in range(1, 200):
        e.save_entry(0, 1, i, fake * 20)
    out.append(("false_candidates", e.getvalue(), 1, False))
    # a metadata conflict late in the WAL (a second metadata record with other bytes)
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"m1")
    for i in range(1, 150):
        e.save_entry(0, 1, i, rng.randbytes(rng.randrange(0, 900)))
        if i == 120:
            e.encode(1, b"m2")
    out.append(("meta_late", e.getvalue(), 1, False))
    # an index gap late in the WAL, a rewind (leader change) late in the WAL
    for kind, jump in (("gap_late", 3), ("rewind_late", -4)):
        e = O.WalEncoder(0)
        e.save_crc(0)
        e.encode(1, b"m")
        idx = 1
        for i in range(150):
            if i == 110:
                idx += jump
            e.save_entry(0, 1 if i < 110 else 2, idx, rng.randbytes(rng.randrange(0, 900)))
            idx += 1
        out.append((kind, e.getvalue(), 1, False))
    # a torn tail, ErrIndexNotFound
    out.append(("torn_tail", w[:-7], 1, False))
    out.append(("index_not_found", w, 10 ** 6, False))
    return out


def _frame0_cases(rng, world):
    """frame 0 of each later range corrupt (its stored CRC / its Data): the
    deferred check must catch it (GPU)"""
    out = []
    w = _wal(rng, cuts=0)
    offs = _frames(w)
    n = len(w)
    for r in range(1, world):
        start = r * n // world
        f0 = next(p for p in offs if p >= start)
        b = bytearray(w)
        b[f0 + 8 + 3] ^= 0x01          # the first byte of the stored CRC varint (08 02 10 <crc>)
        out.append(("frame0_crc_%d" % r, bytes(b), 1, True))
        b = bytearray(w)
        L = struct.unpack_from("<q", w, f0)[0]
        b[f0 + 8 + L - 1] ^= 0x20      # its last Data byte
        out.append(("frame0_data_%d" % r, bytes(b), 1, True))
    return out


def _cpu_probe(buf, start, window=1 << 20):
    """ewal_range_probe's answer from the bytes (test helper)"""
    B = len(buf)
    for p in range(start, min(B, start + window)):
        if p + 11 <= B and buf[p + 8] == 0x08 and buf[p + 9] < 0x80 and buf[p + 10] == 0x10:
            L = struct.unpack_from("<q", buf, p)[0]
            if 4 <= L <= B - p - 8:
                q, idx = p, -1
                for _ in range(64):
                    if q + 8 > B:
                        break
                    L2 = struct.unpack_from("<q", buf, q)[0]
                    if L2 < 0 or q + 8 + L2 > B:
                        break
                    st, r = O.record_unmarshal(buf[q + 8:q + 8 + L2])
                    if st != O.OK:
                        break
                    if r["type"] == 2 and r["data"]:
                        est, e = O.entry_unmarshal(r["data"])
                        if est == O.OK:
                            idx = e["index"]
                        break
                    q += 8 + L2
                return p, idx
    return -1, -1


def _oracle_range(allb, start, end, ri):
    """the range's deferred ReadAll emulated with the oracle: behind a crcType
    record carrying the true running CRC before `start` (frame numbers -1)"""
    buf = allb[start:end]
    if start == end:        # an empty range (joined into an earlier one)
        return (O.OK, -1, 0, 0), oracle_range_info(b"", ri)
    crcs, offs = O.chain_crcs(allb)

    def running_after(o):   # ErrIndexNotFound carries no lastCRC in Go; the range still hands it on
        if o["status"] == O.ERR_INDEX_NOT_FOUND and o["n_records"]:
            last = max(i for i, x in enumerate(offs) if x < end)
            return crcs[last]
        return o["last_crc"]
    if start == 0:
        o = O.readall(buf, ri)
        return (o["status"], o["fail_record"], o["n_records"], running_after(o)), oracle_range_info(buf, ri)
    if start not in offs:   # a false candidate: the range before it is cut short and resplits first
        info = oracle_range_info(b"", ri)
        info["n_bytes"] = end - start
        return (O.ERR_UNEXPECTED_EOF, 0, 0, 0), info
    k = offs.index(start)
    pre = O.WalEncoder(crcs[k - 1])
    pre.save_crc(crcs[k - 1])
    o = O.readall(pre.getvalue() + buf, ri)
    res = (o["status"], o["fail_record"] - 1 if o["fail_record"] >= 0 else -1, o["n_records"] - 1, running_after(o))
    info = oracle_range_info(buf, ri)
    L = struct.unpack_from("<q", buf, 0)[0]
    st, r = O.record_unmarshal(buf[8:8 + L])
    info.update(first_type=r["type"], first_dlen=len(r["data"] or b""), first_stored_crc=r["crc"],
                first_u0=r["crc"] if r["type"] == 4 else O.crc32_update(0, r["data"] or b""),
                first_pre_crc=1 if st != O.OK else 0)
    return res, info


def _worker(rank, world, port, cases, use_gpu, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=180))
    try:
        ctx = None
        if use_gpu:
            from etcd_amd import wal as W
            ctx = W.Context(0)
        out = []
        for kind, allb, rig, _ in cases:
            n = len(allb)
            if use_gpu:
                def probe(start):
                    d = ctx.alloc(n - start + 64)
                    d.upload(allb[start:])
                    try:
                        p, idx = W.range_probe(d, n - start, 0)
                    finally:
                        d.free()
                    return (p + start if p >= 0 else -1), idx
            else:
                def probe(start):
                    return _cpu_probe(allb, start)
            bounds = shard.range_bounds(dist, world, rank, probe, n, rig)
            ranges = [(s, e, ri) for s, e, ri in bounds]
            for _ in range(world + 1):
                s, e, ri = ranges[rank]
                if use_gpu:   # the product alone
                    buf = allb[s:e]
                    d = ctx.alloc(len(buf) + 64)
                    if buf:
                        d.upload(buf)
                    g = W.readall_range_device(d, len(buf), ri, defer_first=s > 0)
                    res = (g.status, g.fail_record, g.n_records, g.last_crc)
                    info = W.range_info(ctx, stream=buf)
                    d.free()
                else:
                    res, info = _oracle_range(allb, s, e, ri)
                v = shard.split_verdict(dist, world, rank, res, info, ri, rig, deferred=s > 0)
                if v[3] < 0:
                    break
                k = v[3]      # ranges k.. verified joined on rank k
                ranges = ranges[:k] + [(ranges[k][0], n, ranges[k][2])] + [(n, n, rig)] * (world - k - 1)
                out.append(("resplit", kind, k))
            out.append((kind,) + tuple(v[:3]))
        if ctx is not None:
            ctx.close()
        q.put((rank, out))
    except Exception:
        q.put((rank, [("error", traceback.format_exc())]))
        raise
    finally:
        dist.destroy_process_group()


def _run(world, use_gpu, cases):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cases, use_gpu, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert not any(x[0] == "error" for x in res[r]), res[r]
        got = [x for x in res[r] if x[0] != "resplit"]
        assert len(got) == len(cases)
        for (kind, allb, rig, _), g in zip(cases, got):
            o = O.readall(allb, rig)
            want = (kind, o["status"], o["fail_record"] if o["status"] not in (O.OK, O.ERR_INDEX_NOT_FOUND) else -1,
                    o["n_records"])
            assert g == want, (r, g, want)
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_within_file_split_oracle_ranges(world):
    cases = _cases(random.Random(31 + world))
    res = _run(world, False, cases)
    # the false candidates made a range start inside a record: found and resplit
    assert any(x[0] == "resplit" and x[1] == "false_candidates" for x in res[0])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_within_file_split_gpu_ranges(world):
    rng = random.Random(41 + world)
    _run(world, True, _cases(rng) + _frame0_cases(rng, world))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_within_file_split_gpu_mutated(world):
    # damaged WALs (test_gpu_fuzz's mutations: flips, torn tails, inserted /
    # deleted bytes, frames duplicated / dropped / swapped) split over the ranks:
    # the joined verdict must still be ReadAll's over the whole WAL
    from test_gpu_fuzz import _mutate
    rng = random.Random(77 + world)
    cases = [("mutated_%d" % i, _mutate(rng, _wal(rng, n=rng.randrange(60, 300), cuts=rng.randrange(0, 3))), 1, True)
             for i in range(16)]
    _run(world, True, cases)
