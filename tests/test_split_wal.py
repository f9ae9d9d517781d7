"""ONE WAL split across ranks by file (each file starts with a
crcType record carrying the running CRC, wal/wal.go:93,232-234): every rank
runs ReadAll over its contiguous range of files, then shard.split_verdict's
one all-gather applies ReadAll's cross-file rules (crc seam, metadata) in file
order.  The global verdict must equal ReadAll over all the files.

CPU (gloo, world_size 2 and 3): each range's result and range info come from
the oracle.  GPU (-m gpu, world_size 2 on one MI355X, gloo for the exchange):
from the product alone -- ReadAll and ewal_copy_range_info (libewal.so); no
oracle parser builds the per-range inputs (the oracle only judges the joined
verdict)."""
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


def build_files(rng, nfiles, md=b"metadata", md_override=None, ents=(5, 60), shift=None):
    """wal.Create + Save + Cut ... as the reference writes them: file k starts
    with crcType{running CRC} and metadataType{md}; returns [(bytes, the index
    in the file's name)].  shift = {k: (name delta, entry delta)}: file k's
    name index and its first entry Index moved (a leader change rewriting
    indexes after a Cut, a gap, a name that disagrees with the entries)."""
    files, prev, idx = [], 0, 0
    for k in range(nfiles):
        e = O.WalEncoder(prev)
        e.save_crc(prev)
        e.encode(1, md_override.get(k, md) if md_override else md)
        dn, de = (shift or {}).get(k, (0, 0))
        name = idx + dn
        idx += de
        for _ in range(rng.randrange(*ents)):
            e.save_entry(0, 1, idx, rng.randbytes(rng.randrange(0, 2000)))
            idx += 1
        e.save_state(1, 1, idx)
        files.append((e.getvalue(), name))
        prev = e.crc
    return files


def oracle_range_info(buf, ri):
    """wal.range_info()'s fields from the oracle's record and entry decoders
    over the range's framable frames (the CPU stand-in for ewal_range_info)."""
    recs, p = [], 0
    while p + 8 <= len(buf):
        L = struct.unpack_from("<q", buf, p)[0]
        if L < 0 or p + 8 + L > len(buf):
            break
        rs, r = O.record_unmarshal(buf[p + 8:p + 8 + L])
        if rs != O.OK:
            break
        recs.append(r)
        p += 8 + L
    first = recs[0] if recs else None
    # where decoder.decode stops (8 bytes with no payload read as io.EOF); frame 0
    # failing in framing / Record.Unmarshal (before decoder.decode's CRC check)
    end_off = p
    pre = bool(buf) and not recs
    info = dict(n_frames=len(recs), first_crc=recs[0]["crc"] if recs and recs[0]["type"] == 4 else -1,
                first_type=first["type"] if first else -1, first_dlen=len(first["data"] or b"") if first else 0,
                first_stored_crc=first["crc"] if first else 0,
                first_u0=(first["crc"] if first["type"] == 4 else O.crc32_update(0, first["data"] or b"")) if first
                else 0,
                md_first_frame=-1, md_first=None, md_value_frame=-1, md_value=None, first_entry_frame=-1,
                first_entry_index=0, min_entry_index=0, last_entry_index=0, last_op_frame=-1, last_op_index=0,
                last_entry_frame=-1, first_pre_crc=1 if pre else 0, end_off=end_off, n_bytes=len(buf),
                state_frame=-1, state=(0, 0, 0), state_unrec=0)
    idx = []
    for i, r in enumerate(recs):
        if r["type"] == 3:   # the range's last HardState
            _, h = O.hardstate_unmarshal(r["data"] or b"")
            info.update(state_frame=i, state=(h["term"], h["vote"], h["commit"]), state_unrec=int(bool(h["unrec"])))
        if r["type"] == 1:
            if info["md_first_frame"] < 0:
                info["md_first_frame"], info["md_first"] = i, r["data"] or None
            if r["data"] and info["md_value_frame"] < 0:
                info["md_value_frame"], info["md_value"] = i, r["data"]
        elif r["type"] == 2:
            est, e = O.entry_unmarshal(r["data"] or b"")
            idx.append((i, e["index"]))
    if idx:
        info.update(first_entry_frame=idx[0][0], first_entry_index=idx[0][1],
                    min_entry_index=min(x for _, x in idx), last_entry_index=idx[-1][1], last_entry_frame=idx[-1][0])
        ops = [(i, x) for i, x in idx if x >= ri]
        if ops:
            info.update(last_op_frame=ops[-1][0], last_op_index=ops[-1][1])
    return info


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
        for ranges, rig in cases:
            ranges = list(ranges)
            while True:
                buf, ri = ranges[rank]
                if use_gpu:    # the product alone: ReadAll + ewal_range_info over the range
                    g = W.readall_bytes(buf, ri, ctx, with_ents=True)
                    res = (g.status, g.fail_record, g.n_records, g.last_crc)
                    mine = g.as_dict()["ents"] if g.status == O.OK else []
                    info = W.range_info(ctx, stream=buf)
                else:
                    o = O.readall(buf, ri)
                    res = (o["status"], o["fail_record"], o["n_records"], o["last_crc"])
                    mine = o["ents"] if o["status"] == O.OK else []
                    info = oracle_range_info(buf, ri)
                full = shard.split_verdict(dist, world, rank, res, info, ri, rig, full=True)
                v = (full["status"], full["fail_record"], full["n_records"], full["resplit"])
                if v[3] < 0:
                    break
                # ranges k.. verified joined, on rank k
                k = v[3]
                ranges = ranges[:k] + [(b"".join(b for b, _ in ranges[k:]), ranges[k][1])] + \
                    [(b"", 0)] * (world - k - 1)
                out.append(("resplit", k))
            full["ents"] = mine
            out.append((v[:3], full))
        if ctx is not None:
            ctx.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


KINDS = ("clean", "corrupt_late", "corrupt_both", "seam", "meta", "meta_nil", "torn", "dangling", "rewind",
         "gap_cross", "gap_name", "name_low", "index_not_found", "ri_mid")


def _cases(rng, world):
    """[(all bytes, w.ri of the whole ReadAll, [per-rank (range bytes, ri)])]
    over clean / corrupt / seam / metadata-conflict / torn / index-rule WALs."""
    out = []
    for kind in KINDS:
        nf = world * 2
        per = nf // world
        over = {nf // 2: b"other"} if kind == "meta" else ({1: None} if kind == "meta_nil" else None)
        shift = {"rewind": {per: (0, -3)},          # a range's first entries rewrite indexes below its name
                 "gap_cross": {per: (2, 2)},        # name and entries skip two indexes: a gap only globally
                 "gap_name": {per: (0, 2)},         # entries skip two indexes after the name: a gap everywhere
                 "name_low": {per: (-2, 0)}}.get(kind)   # the name lies below the entries: a gap only locally
        files = build_files(rng, nf, md_override=over, shift=shift)
        blobs = [bytearray(b) for b, _ in files]
        if kind == "corrupt_late":
            blobs[-1][len(blobs[-1]) // 2] ^= 0x10
        if kind == "corrupt_both":
            blobs[0][len(blobs[0]) - 30] ^= 0x10
            blobs[-1][len(blobs[-1]) // 2] ^= 0x10
        if kind == "seam":     # the crcType record of the file opening the last range carries a wrong CRC
            k = nf - 2
            b2 = O.WalEncoder(12345)
            b2.save_crc(12345)
            body = bytes(blobs[k])[8 + blobs[k][0]:]
            blobs[k] = bytearray(b2.getvalue() + body)
        if kind == "torn":          # the last file of range 0 torn: its frame reads on into range 1
            blobs[per - 1] = blobs[per - 1][:-5]
        if kind == "dangling":      # range 0 ends with a bare length prefix (io.EOF alone; whole,
            blobs[per - 1] += struct.pack("<q", 40)   # the frame reads its payload from the next file)
        rig = 0
        if kind == "index_not_found":    # OpenAtIndex past the last entry: the global ErrIndexNotFound
            rig = files[-1][1] + 1000
        if kind == "ri_mid":             # OpenAtIndex inside the first file
            rig = 3
        ranges = []
        for r in range(world):
            part = b"".join(bytes(x) for x in blobs[r * per:(r + 1) * per])
            ranges.append((part, rig if r == 0 else max(rig, files[r * per][1])))
        out.append((b"".join(bytes(x) for x in blobs), rig, ranges))
    return out


def _mutated_cases(rng, world, n=12):
    """WALs of world * 2 files with one file damaged by test_gpu_fuzz's
    mutations (flips, torn tails, inserted / deleted bytes, frames
    duplicated / dropped / swapped), split by file over the ranks."""
    from test_gpu_fuzz import _mutate
    out = []
    for _ in range(n):
        nf = world * 2
        per = nf // world
        files = build_files(rng, nf, ents=(3, 30))
        blobs = [bytes(b) for b, _ in files]
        k = rng.randrange(nf)
        blobs[k] = _mutate(rng, blobs[k])
        ranges = [(b"".join(blobs[r * per:(r + 1) * per]), 0 if r == 0 else files[r * per][1]) for r in range(world)]
        out.append((b"".join(blobs), 0, ranges))
    return out


def _run(world, use_gpu, cases=None):
    rng = random.Random(17 + world)
    labels = KINDS if cases is None else tuple("mutated_%d" % i for i in range(len(cases)))
    plain = cases is None
    cases = _cases(rng, world) if plain else cases
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, [(c[2], c[1]) for c in cases], use_gpu, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        got = [x for x in res[r] if x[0] != "resplit"]
        assert len(got) == len(cases)
        if plain:
            assert any(x[0] == "resplit" for x in res[r])   # the torn-file case went through a resplit
        for i, (allb, rig, _) in enumerate(cases):
            o = O.readall(allb, rig)
            want = (o["status"], o["fail_record"] if o["status"] not in (O.OK, O.ERR_INDEX_NOT_FOUND) else -1,
                    o["n_records"])
            assert got[i][0] == want, (labels[i], r, got[i][0], want)
            if o["status"] != O.OK:
                continue
            # the rest of ReadAll's result: metadata, HardState, ents stitched from every rank's
            f = got[i][1]
            assert (f["last_crc"], f["enti"], f["metadata"]) == (o["last_crc"], o["enti"], o["metadata"]), labels[i]
            st = o["state"]
            assert (f["state"] or (0, 0, 0)) == (st["term"], st["vote"], st["commit"]), labels[i]
            assert f["n_ents"] == len(o["ents"]), labels[i]
            joined = []
            for k in range(world):
                b, c = f["layout"][k]
                if c > 0:
                    rk = [x for x in res[k] if x[0] != "resplit"][i][1]["ents"]
                    joined = joined[:b] + rk[:c]
            assert joined == o["ents"], labels[i]
    return cases


@pytest.mark.parametrize("world", [2, 3])
def test_split_verdict_oracle_ranges(world):
    cases = _run(world, use_gpu=False)
    kinds = [O.readall(c[0], c[1])["status"] for c in cases]
    for st in (O.ERR_WAL_CRC, O.ERR_METADATA_CONFLICT, O.ERR_RECORD_CRC, O.PANIC_INDEX_GAP, O.ERR_INDEX_NOT_FOUND):
        assert st in kinds, st


@pytest.mark.gpu
def test_split_verdict_gpu_ranges():
    _run(2, use_gpu=True)


@pytest.mark.parametrize("world", [2, 3])
def test_split_verdict_mutated_oracle_ranges(world):
    _run(world, False, _mutated_cases(random.Random(300 + world), world))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_split_verdict_mutated_gpu_ranges(world):
    _run(world, True, _mutated_cases(random.Random(400 + world), world))


@pytest.mark.gpu
def test_range_info_gpu_matches_oracle(ctx):
    """ewal_copy_range_info field by field against the oracle's decoders, on
    every range of every split case (world 2 and 3)."""
    from etcd_amd import wal as W
    for world in (2, 3):
        for allb, rig, ranges in _cases(random.Random(17 + world), world):
            for buf, ri in ranges + [(allb, rig)]:
                g = W.readall_bytes(buf, ri, ctx, with_ents=False)
                o = O.readall(buf, ri)
                assert (g.status, g.fail_record, g.n_records) == (o["status"], o["fail_record"], o["n_records"])
                gi, oi = W.range_info(ctx, stream=buf), oracle_range_info(buf, ri)
                if g.status == O.OK:      # every frame framable: the chain is the oracle's frame list
                    assert gi == oi, (gi, oi)
                else:                     # the fields split_verdict reads before the failure
                    for key in ("first_crc", "md_first_frame", "md_first", "first_entry_frame", "first_entry_index"):
                        if oi["md_first_frame"] < g.fail_record or not key.startswith("md"):
                            assert gi[key] == oi[key], (key, gi[key], oi[key])
