#!/usr/bin/env python3
"""bench.py -- etcd WAL replay-and-verify on MI355X (BASELINE.json metric).

Default line (value, ms_per_step, roofline, cpu_baseline): configs[1] -- one
step = one (*WAL).ReadAll (wal/wal.go:164-216) over a GPU-resident synthetic
WAL of 8 GiB of mixed 64 B - 64 KiB entries (log-uniform sizes, xorshift
payload) with one corrupt record at frame k = 0.73 N, so every step must
report walpb.ErrCRCMismatch at frame k.  The whole WAL is read and verified
each step (the GPU pipeline does not stop early).  The same line carries
`configs`: every other BASELINE config timed in the same run, each with its
own ms_per_step, roofline and (N=1) cpu_baseline --
  c1      configs[0]: the 1M x 256 B WAL (wal.Save) replayed on the GPU
  shards  configs[2]: 512 per-raft-group WALs x 64 MiB per GPU (4096 over
          8 GPUs), one batched ReadAll per step, one RCCL all-reduce
  snap    configs[3]: a resident batch of snapshot files, loadSnap's CRC
  snapstream configs[3] at its full size: the 10k-file set (~450 GiB, 1-256
          MiB) streamed from pinned host memory through two HBM batches
  commit  configs[4]: maybeCommit over 1M raft groups x 5/7 voters
  rewind  the configs[1]-shaped WAL after leader changes (1 % of the entries
          rewrite the last 1-8 indexes): ReadAll's rewind path timed
With --gpus N (torchrun) every rank verifies its own independent shards
(weak scaling) and one RCCL all-reduce per step combines the verdicts.

Prints ONE JSON line on rank 0 (value = GB/s over all ranks, 1 GB = 1e9 B).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: its HIP runtime is the one libewal.so binds to)
from etcd_amd import wal as W, _lib as L, shard  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size-gib", type=float, default=8.0)
    ap.add_argument("--min-data", type=int, default=64)
    ap.add_argument("--max-data", type=int, default=65536)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--snap-files", type=int, default=10000)
    ap.add_argument("--pool-gib", type=float, default=None,
                    help="snapstream's pinned host pool per rank (default 24 GiB at N=1, max(6, 48 / N) at N>1: "
                         "the files are drawn from it at random, so its size does not move the PCIe-bound rate, and "
                         "8 ranks x 24 GiB of pinned memory would be 192 GiB of the node's RAM)")
    ap.add_argument("--batch-gib", type=float, default=8.0)
    ap.add_argument("--workload", choices=["wal", "c1", "shards", "snap", "snapstream", "commit", "msg", "restart",
                                           "rewind"],
                    default="wal",
                    help="wal = configs[1] (the headline, default); c1 = configs[0]'s WAL (1M x 256 B entries) on "
                         "the GPU; shards = configs[2] (4096 x 64 MiB per-group WALs over the node, 512 per GPU); "
                         "snap = configs[3] (a resident batch); snapstream = configs[3]'s 10k-file set streamed "
                         "from pinned host memory; commit = configs[4]; msg = raftpb.Message ingress decode; "
                         "restart = OpenAtIndex + ReadAll + materialise through the C ABI (the cgo shim's calls)")
    ap.add_argument("--shards-per-gpu", type=int, default=512)
    ap.add_argument("--shard-mib", type=int, default=64)
    ap.add_argument("--configs", default="c1,shards,snap,snapstream,commit,rewind,split2",
                    help="default line: the other BASELINE configs timed in the same run ('none' to skip)")
    ap.add_argument("--sub-cpu-seconds", type=float, default=6.0,
                    help="CPU-baseline time per leg of each `configs` sub-result")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL; gloo only to rehearse the N>1 path)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on cuda:0 (with --dist-backend gloo)")
    return ap.parse_args()


def load_traffic(kernel="k_stream", workload=None):
    """Per-launch HBM bytes of a kernel from its committed PMC pass at this
    workload, if any (profiles/<kernel>_pmc[_<workload>].json, tools/traffic.sh
    + tools/traffic.py)."""
    p = os.path.join(ROOT, "profiles", kernel + "_pmc" + ("_" + workload if workload else "") + ".json")
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


METRIC = "WAL verify GB/s (and records/s) per GPU + 8-GPU node, % of HBM roofline"


CPU_SHARE = 16   # the GPU box's CPU share per GPU (nproc / the CPU set show the whole machine's)


def cpu_threads():
    """The host cores the CPU baselines may use: the process's CPU set,
    capped at the box's per-GPU share of 16 CPUs."""
    return max(1, min(CPU_SHARE, len(os.sched_getaffinity(0))))


def host_info():
    """Recorded with every cpu_baseline (BASELINE.md:29)."""
    import shutil
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    go = shutil.which("go")
    return {"cpu_model": model, "nproc": os.cpu_count(), "cpus_allowed": len(os.sched_getaffinity(0)),
            "cores_note": "multi-core legs use min(cpus_allowed, %d): the GPU box's CPU share per GPU, not every "
                          "CPU of the host" % CPU_SHARE,
            "gomaxprocs": "n/a (no Go toolchain on this host; the C restatement is timed instead)" if not go else
                          "n/a (go at %s not used: the reference is not built here)" % go}


def timed_cpu(seconds, fn):
    """Run fn until `seconds` have passed (at least once): (passes, elapsed)."""
    it, t0 = 0, time.perf_counter()
    while True:
        fn()
        it += 1
        if time.perf_counter() - t0 >= seconds:
            return it, time.perf_counter() - t0


def timed(dist, steps, fn):
    """barrier + sync, K steps, sync + barrier; the max over ranks (s)."""
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed


# k_frames' algorithmic bytes: per frame its 80-B head read and
# its 40-B ewal_entry written (every synthetic frame but the 3 head frames is
# an entry op), per 4 KiB unit its 64 B of v[] and 16 B of hmask read and 8 B
# (pl, ucb) written.
FR_FRAME_B, FR_UNIT_B = 80 + 40, 64 + 16 + 8


def frames_roofline(frames, nbytes, kernel_ms, workload):
    if not kernel_ms:
        return None
    ab = frames * FR_FRAME_B + (nbytes // 4096 + 1) * FR_UNIT_B
    ach = ab / (kernel_ms / 1e3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4), "kernel": "k_frames", "kernel_ms": round(kernel_ms, 4),
            "algorithmic_bytes_per_launch": int(ab),
            "bytes_model": "per frame 80-B head + 40-B entry, per 4 KiB unit 64-B v[] + 16-B hmask + 8 B out",
            "traffic": load_traffic("k_frames", workload),
            "traffic_source": "profiles/k_frames_pmc_%s.json (a committed PMC pass of this workload; null: none)" % workload,
            "note": "the frame pass is issue- and latency-bound (profiles/r05/sq_counters_k_stream_k_frames.txt), "
                    "not HBM-bound: its fraction is low by construction"}


def run_shards(a, dist, rank, world, local, cpu_seconds=None):
    """configs[2]: 4096 per-raft-group WAL shards x 64 MiB over the node --
    each GPU replays its 512 (at N=8) in ONE batched ReadAll
    (ewal_readall_batch_device); entries 128 B - 4 KiB log-uniform, seed =
    global shard id; one corrupt record in global shard 2749 mod (512 N).
    The verdicts cross ranks in one all-reduce (etcd_amd/shard.py).  The
    shards are generated and copied to HBM 64 at a time (host memory stays
    at ~4 GiB per rank).  `torn5`: the same batch with the last frame of 5
    shards torn (a crash mid-write): the batch's own pass classifies their
    terminal (wal/decoder.go:30-36), no shard is replayed alone.  `rew1pct`:
    1 % of the shards replaced by WALs after leader changes (index rewinds,
    wal/wal.go:170-176), decided by the batch's rewind-mode pass."""
    nsh, smib = a.shards_per_gpu, a.shard_mib
    cpu_seconds = a.cpu_seconds if cpu_seconds is None else cpu_seconds
    first = rank * nsh
    bad_shard = 2749 % (nsh * world)
    t = time.time()
    target = smib << 20
    chunk = 64
    ctx = W.Context(local)
    dev = torch.device("cuda", local)
    dmem = torch.empty(nsh * (target + (1 << 20)) + 64, dtype=torch.uint8, device=dev)   # (the generator overshoots)
    dbuf = W.DeviceBuffer(ctx, C.c_void_p(dmem.data_ptr()), dmem.numel())   # torch owns it
    lens, nrec, pos, keep = [], [], 0, None
    for c0 in range(0, nsh, chunk):
        ids = list(range(c0, min(nsh, c0 + chunk)))
        blob, ls, nr = W.synth_shards([first + i for i in ids], target, 128, 4096,
                                      corrupt={bad_shard - first - c0: 1000}
                                      if first + c0 <= bad_shard < first + c0 + len(ids) else {})
        dmem[pos:pos + len(blob)].copy_(torch.frombuffer(blob, dtype=torch.uint8))
        pos += len(blob)
        lens += ls
        nrec += nr
        if c0 == 0:
            keep = blob     # the CPU baseline's sample
        del blob
    gen_s = time.time() - t
    nb = pos
    ris = [1] * nsh
    res = None
    for _ in range(max(a.warmup, 1)):
        res = W.readall_batch_device(dbuf, lens, ris)
    for i, r in enumerate(res):
        want = (L.ERR_RECORD_CRC, 1000) if first + i == bad_shard else (L.OK, -1)
        assert (r.status, r.fail_record) == want and not (r.flags & L.FLAG_SHARD_FALLBACK), (i, r.status, r.flags)
        assert r.status != L.OK or r.n_records == nrec[i]
    summary = torch.zeros(3, dtype=torch.int64, device="cuda") if dist is not None else None
    last = {}

    # the C ABI straight into preallocated arrays: no per-shard Python objects in the timed region
    c_lens, c_ris = (C.c_uint64 * nsh)(*lens), (C.c_uint64 * nsh)(*ris)
    c_out = (L.Result * nsh)()

    def step():
        rc = L.lib.ewal_readall_batch_device(ctx.handle, dbuf.ptr, nsh, c_lens, c_ris, c_out)
        assert rc == 0, rc
        last["r"] = c_out
        if dist is not None:   # one all-reduce of the batch's verdicts (etcd_amd/shard.py)
            last["v"] = shard.combine_batch(dist, first, [(x.fail_record if x.status != L.OK else -1, x.n_records,
                                                           x.status != L.OK) for x in c_out], out=summary)

    fr_ms = []

    def step_t():
        step()
        fr_ms.append(c_out[0].frames_ms)

    elapsed = timed(dist, a.steps, step_t)
    ms = elapsed / a.steps * 1e3
    r0 = L.Result.from_buffer_copy(last["r"][0])   # (c_out is reused below)
    frames_ms = sum(fr_ms) / len(fr_ms)
    assert all((x.status, x.fail_record) == ((L.ERR_RECORD_CRC, 1000) if first + i == bad_shard else (L.OK, -1))
               for i, x in enumerate(c_out))
    frames = sum(nrec)
    # the node's verdict: the all-reduced {MIN first-corrupt key, SUM frames, SUM failing shards} of the last
    # step (N = 1: the same reduction over this rank's shards), and every rank's kernel times
    if dist is not None:
        key, vframes, vfail = last["v"]
        kt = torch.tensor([r0.stream_ms, frames_ms, r0.device_ms, float(nb), float(frames)], dtype=torch.float64,
                          device="cuda")
        allk = [torch.zeros_like(kt) for _ in range(world)]
        dist.all_gather(allk, kt)
        per_rank = [dict(rank=i, stream_ms=round(float(x[0]), 4), frames_ms=round(float(x[1]), 4),
                         pipeline_ms=round(float(x[2]), 4),
                         roofline_frames=frames_roofline(int(x[4]), int(x[3]), float(x[1]), "shards"))
                    for i, x in enumerate(allk)]
    else:
        key, vframes, vfail = shard.combine_batch_local(first, [(x.fail_record if x.status != L.OK else -1,
                                                                 x.n_records, x.status != L.OK) for x in c_out])
        per_rank = None
    dk = shard.decode_key(key)
    assert dk == (bad_shard, 1000) and vfail == 1, (dk, vfail)
    verdict = {"first_corrupt": {"shard": dk[0], "frame": dk[1]}, "frames_verified": vframes,
               "failing_shards": vfail,
               "note": "all-reduced over the ranks (MIN first-corrupt key = shard << 40 | frame, SUM frames, "
                       "SUM failing shards), the last timed step's"}
    # ---- torn5: five shards end in a torn frame -----------------------------
    torn = sorted({(nsh * j) // 5 + 7 for j in range(5)} - {bad_shard - first})[:5]
    tlens = [x - (1000 + 37 * i) if i in torn else x for i, x in enumerate(lens)]
    tmem = torch.empty(sum(tlens) + 64, dtype=torch.uint8, device=dev)
    so, to = 0, 0
    for x, y in zip(lens, tlens):
        tmem[to:to + y].copy_(dmem[so:so + y])
        so += x
        to += y
    tbuf = W.DeviceBuffer(ctx, C.c_void_p(tmem.data_ptr()), tmem.numel())
    c_tlens = (C.c_uint64 * nsh)(*tlens)
    torch.cuda.synchronize()

    def tstep():
        rc = L.lib.ewal_readall_batch_device(ctx.handle, tbuf.ptr, nsh, c_tlens, c_ris, c_out)
        assert rc == 0, rc

    for _ in range(max(a.warmup, 1)):
        tstep()
    for i, x in enumerate(c_out):
        if i in torn:
            assert x.status == L.ERR_UNEXPECTED_EOF and not x.flags & L.FLAG_SHARD_FALLBACK, (i, x.status, x.flags)
        else:
            want = (L.ERR_RECORD_CRC, 1000) if first + i == bad_shard else (L.OK, -1)
            assert (x.status, x.fail_record) == want and not x.flags & L.FLAG_SHARD_FALLBACK, (i, x.status)
    tms = timed(dist, a.steps, tstep) / a.steps * 1e3
    torn5 = {"ms_per_step": round(tms, 4), "vs_clean": round(tms / ms, 4), "torn_shards": torn,
             "note": "the same batch with the last frame of 5 shards torn: the batch's fused pass gives "
                     "their verdict (io.ErrUnexpectedEOF at the torn frame), no shard is replayed alone"}
    del tmem
    # ---- rew1pct: 1 % of the shards after leader changes (index rewinds) ----
    nrw = max(1, nsh // 100)
    rws = sorted({(nsh * j) // nrw + 11 for j in range(nrw)} - {bad_shard - first})[:nrw]
    rblobs, rli = {}, {}
    for i in rws:
        li = []
        b, _ = W.synth_wal(target, 128, 4096, seed=700000 + first + i, rewind_per_mille=10, last_index=li)
        rblobs[i], rli[i] = b, li[0]
    rlens = [len(rblobs[i]) if i in rblobs else x for i, x in enumerate(lens)]
    rmem = torch.empty(sum(rlens) + 64, dtype=torch.uint8, device=dev)
    so, to = 0, 0
    for i, (x, y) in enumerate(zip(lens, rlens)):
        if i in rblobs:
            rmem[to:to + y].copy_(torch.frombuffer(rblobs[i], dtype=torch.uint8))
        else:
            rmem[to:to + y].copy_(dmem[so:so + y])
        so += x
        to += y
    del rblobs
    rbuf = W.DeviceBuffer(ctx, C.c_void_p(rmem.data_ptr()), rmem.numel())
    c_rlens = (C.c_uint64 * nsh)(*rlens)
    torch.cuda.synchronize()

    def rstep():
        rc = L.lib.ewal_readall_batch_device(ctx.handle, rbuf.ptr, nsh, c_rlens, c_ris, c_out)
        assert rc == 0, rc

    for _ in range(max(a.warmup, 1)):
        rstep()
    for i, x in enumerate(c_out):
        assert not x.flags & L.FLAG_SHARD_FALLBACK, (i, x.status, x.flags)
        if i in rli:
            assert x.status == L.OK and x.n_ents == rli[i], (i, x.status, x.n_ents, rli[i])
        else:
            want = (L.ERR_RECORD_CRC, 1000) if first + i == bad_shard else (L.OK, -1)
            assert (x.status, x.fail_record) == want, (i, x.status)
    rwms = timed(dist, a.steps, rstep) / a.steps * 1e3
    rew1pct = {"ms_per_step": round(rwms, 4), "vs_clean": round(rwms / ms, 4), "rewinding_shards": rws,
               "note": "the same batch with %d shards (1 %%) replaced by WALs after leader changes (1 %% of their "
                       "entries rewrite the last 1-8 indexes, wal/wal.go:170-176): no shard is replayed alone; "
                       "the ctx's previous batch of this shape saw those shards rewind, so the batch's own frame "
                       "pass runs them in rewind mode (slot claims + k_ents_fix, no second pass; the first call "
                       "of a shape reruns the claims over their tiles, k_rew_claim)" % len(rws)}
    del rmem
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # baseline only
        nth = cpu_threads()
        k = min(chunk, nsh)              # a bounded sample: the first chunk of shards
        so = [0]
        for x in lens[:k - 1]:
            so.append(so[-1] + x)
        sl = lens[:k]
        sb = sum(sl)
        addr = C.addressof((C.c_char * len(keep)).from_buffer(keep))
        it, cs = timed_cpu(cpu_seconds, lambda: O.fast_readall_batch(addr, so, sl, 1, nth, faithful=True))
        it2, cs2 = timed_cpu(cpu_seconds / 2, lambda: O.fast_readall_batch(addr, so, sl, 1, nth))
        st, fr = O.fast_readall_batch(addr, so, sl, 1, nth)
        assert all(x in (O.OK, O.ERR_RECORD_CRC) for x in st), st
        cpu = dict(host_info(), **{
            "value": round(sb * it / cs / 1e9, 4), "unit": "GB/s", "cores": nth, "kind": "port",
            "sample": "oracle/ or_readall (the faithful C restatement of wal.ReadAll) on %d cores, one shard per "
                      "worker, over the first %d shards (%.2f GiB), %d passes, %.1f s" % (nth, k, sb / (1 << 30), it, cs),
            "optimised": {"value": round(sb * it2 / cs2 / 1e9, 4), "unit": "GB/s", "cores": nth,
                          "sample": "oracle/ewal_cpu_fast.c orf_readall (3-stream SSE4.2 CRC-32C, no per-record "
                                    "allocation) one shard per worker, same shards, %d passes, %.1f s" % (it2, cs2)}})
    del keep
    out = {
        "metric": METRIC, "value": round(world * nb / (ms / 1e3) / 1e9, 3), "unit": "GB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "configs[2]: %d per-raft-group WAL shards x %d MiB per GPU (%d on 8 GPUs), entry "
                               "Data log-uniform 128 B-4 KiB, seed = shard id, one corrupt record in shard %d; one "
                               "batched ReadAll per GPU per step" % (nsh, smib, nsh * 8, bad_shard),
                   "wal_bytes_per_gpu": nb, "frames_per_gpu": frames, "shards_per_gpu": nsh, "ri": 1,
                   "parallelism": "dp%d (independent shards, one all-reduce of verdicts)" % world},
        "records_per_s": round(world * frames / (ms / 1e3), 1),
        "roofline": {"bound": "hbm", "achieved": round(nb / (r0.stream_ms / 1e3) / 1e9, 2),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(nb / (r0.stream_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": "k_stream", "kernel_ms": round(r0.stream_ms, 4),
                     "algorithmic_bytes_per_launch": nb,
                     "pipeline_achieved": round(nb / (r0.device_ms / 1e3) / 1e9, 2),
                     "pipeline_frac": round(nb / (r0.device_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "step_frac": round(nb / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "pipeline_device_ms": round(r0.device_ms, 4),
        "post_stream_ms": round(r0.post_ms, 4),
        "roofline_frames": frames_roofline(frames, nb, frames_ms, "shards"),
        "verdict": verdict,
        "per_rank": per_rank,
        "torn5": torn5,
        "rew1pct": rew1pct,
        "cpu_baseline": cpu,
        "gen_seconds": round(gen_s, 2),
    }
    del dmem
    ctx.close()
    return out


def run_snap(a, dist, rank, world, local, cpu_seconds=None):
    """configs[3]: batch verification of snap/snapshotter snapshot files
    (loadSnap's CRC, snap/snapshotter.go:76-111): sizes log-uniform 1-256 MiB
    (seed 4), ~1 % corrupt (seed 5, at least one).  The 10k-file set is
    ~450 GiB, more than one GPU holds: each GPU verifies a resident batch of
    16 GiB (--size-gib when given) per step in ONE esnap_verify_packed call
    (8 GPUs: ~56 GiB each).  Files go to HBM as they are made (host memory
    stays at one file plus the CPU baseline's ~1 GiB sample)."""
    import math
    import random
    import numpy as np
    from etcd_amd import snap as S
    cpu_seconds = a.cpu_seconds if cpu_seconds is None else cpu_seconds
    rng, crng = random.Random(4 + 7919 * rank), random.Random(5 + 7919 * rank)
    budget = int((a.size_gib if a.size_gib != 8.0 else 16.0) * (1 << 30))
    t = time.time()
    pool = np.random.default_rng(4 + rank).integers(0, 256, size=(256 << 20) + 4096, dtype=np.uint8).tobytes()
    ctx = W.Context(local)
    dbuf = ctx.alloc(budget + (257 << 20))
    lens, bad, total, sample = [], [], 0, {}
    while total < budget:
        n = int(math.exp(rng.uniform(math.log(1 << 20), math.log(256 << 20))))
        st = rng.randrange(0, len(pool) - n)
        f = bytearray(S.snap_file(S.snapshot_marshal(pool[st:st + n], (1, 2, 3), len(lens) + 1, 1)))
        if crng.random() < 0.01 or (not bad and total + len(f) >= budget):
            f[len(f) // 2] ^= 0x10      # inside Data: snap.ErrCRCMismatch
            bad.append(len(lens))
        dbuf.upload(f, total)
        if len(f) <= (8 << 20) and sum(len(x) for x in sample.values()) < (1 << 30):
            sample[len(lens)] = bytes(f)   # the CPU baseline's sample: the small files, up to 1 GiB
        lens.append(len(f))
        total += len(f)
    del pool
    offs = [0]
    for x in lens[:-1]:
        offs.append(offs[-1] + x)
    gen_s = time.time() - t
    nb = total
    for _ in range(max(a.warmup, 1)):
        stt, _, _ = S.verify_packed(dbuf, nb, offs, lens)
    assert [i for i, x in enumerate(stt) if x != L.OK] == bad and all(stt[i] == L.ERR_SNAP_CRC for i in bad), bad
    last = {}

    def step():
        last["st"] = S.verify_packed(dbuf, nb, offs, lens)[0]

    elapsed = timed(dist, a.steps, step)
    assert [i for i, x in enumerate(last["st"]) if x != L.OK] == bad
    ms = elapsed / a.steps * 1e3
    kms = float(L.lib.ewal_last_stream_ms(ctx.handle))
    dev_ms = float(L.lib.ewal_last_device_ms(ctx.handle))
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # baseline only
        views = list(sample.values())
        acc = sum(len(v) for v in views)

        def one_pass():
            for v in views:
                O.loadsnap(v)
        it, cs = timed_cpu(cpu_seconds, one_pass)
        nth = cpu_threads()
        blob = b"".join(views)
        so = [0]
        for v in views[:-1]:
            so.append(so[-1] + len(v))
        sl = [len(v) for v in views]
        addr = C.cast(C.c_char_p(blob), C.c_void_p).value   # blob's own bytes (no copy)
        it2, cs2 = timed_cpu(cpu_seconds / 2, lambda: O.fast_snap_verify_batch(addr, so, sl, nth))
        st2, _ = O.fast_snap_verify_batch(addr, so, sl, nth)
        assert [k for k, x in zip(sample, st2) if x != O.OK] == [k for k in sample if k in bad]
        cpu = dict(host_info(), **{
            "value": round(acc * it / cs / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle/ or_loadsnap (snappb + raftpb.Snapshot Unmarshal, crc32.Update, 1 thread) over "
                      "%d of the files (<= 8 MiB each, %.2f GiB), %d passes, %.1f s" % (len(views), acc / (1 << 30),
                                                                                       it, cs),
            "optimised": {"value": round(acc * it2 / cs2 / 1e9, 4), "unit": "GB/s", "cores": nth,
                          "sample": "oracle/ewal_cpu_fast.c orf_snap_verify_batch (envelope + 3-stream SSE4.2 "
                                    "CRC-32C) one file per worker over the same files, %d passes, %.1f s"
                                    % (it2, cs2)}})
    out = {
        "metric": METRIC, "value": round(world * nb / (ms / 1e3) / 1e9, 3), "unit": "GB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "configs[3]: snapshot batch verify, %d files per GPU (%.2f GiB resident), sizes "
                               "log-uniform 1-256 MiB, %d corrupt (snap.ErrCRCMismatch)" %
                               (len(lens), nb / (1 << 30), len(bad)),
                   "snapshot_bytes_per_gpu": nb, "files_per_gpu": len(lens),
                   "parallelism": "dp%d (independent files)" % world},
        "files_per_s": round(world * len(lens) / (ms / 1e3), 1),
        "roofline": {"bound": "hbm", "achieved": round(nb / (kms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(nb / (kms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": "k_stream<false>", "kernel_ms": round(kms, 4),
                     "algorithmic_bytes_per_launch": nb,
                     "pipeline_achieved": round(nb / (dev_ms / 1e3) / 1e9, 2),
                     "pipeline_frac": round(nb / (dev_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "pipeline_device_ms": round(dev_ms, 4),
        "cpu_baseline": cpu, "gen_seconds": round(gen_s, 2)}
    dbuf.free()
    ctx.close()
    return out


def run_snapstream(a, dist, rank, world, local, cpu_seconds=None):
    """configs[3] at its full size on one GPU: the 10k-file snapshot set
    (~450 GiB, sizes log-uniform 1-256 MiB) streamed from pinned host
    memory through two HBM batch buffers: the H2D copies of batch b+1 (a
    copy stream) overlap the verification of batch b (esnap_verify_packed,
    snap/snapshotter.go:76-111).  The files are drawn (seed 6) from a pool
    of distinct procedurally generated files held in pinned memory (the
    host holds ~270 GiB at most, not 450 GiB), ~1 % of them corrupt; every
    file of the stream is copied and verified.  value = streamed GB/s
    (host-resident pinned -> verdict); the line also carries the resident
    (kernel-only) rate over the same batches."""
    import math
    import random
    import numpy as np
    from etcd_amd import snap as S
    nfiles = a.snap_files
    rng, crng, prng = random.Random(4 + 7919 * rank), random.Random(5 + 7919 * rank), random.Random(6 + 7919 * rank)
    t = time.time()
    src = np.random.default_rng(4 + rank).integers(0, 256, size=(256 << 20) + 4096, dtype=np.uint8).tobytes()
    sizes, total = [], 0
    pool_gib = a.pool_gib if a.pool_gib is not None else (24.0 if world == 1 else max(6.0, 48.0 / world))
    budget = int(pool_gib * (1 << 30))
    while total < budget:
        n = int(math.exp(rng.uniform(math.log(1 << 20), math.log(256 << 20))))
        sizes.append(n + 64)    # + the snappb / raftpb.Snapshot envelope (upper bound)
        total += n + 64
    pool = torch.empty(total + 16 * len(sizes) + 4096, dtype=torch.uint8).pin_memory()
    pv = pool.numpy()
    poffs, plens, pbad = [], [], []
    pos = 0
    for i, n in enumerate(sizes):
        st = rng.randrange(0, len(src) - n)
        f = bytearray(S.snap_file(S.snapshot_marshal(src[st:st + n - 64], (1, 2, 3), i + 1, 1)))
        if crng.random() < 0.01 or (i == len(sizes) - 1 and not pbad):
            f[len(f) // 2] ^= 0x10
            pbad.append(i)
        pv[pos:pos + len(f)] = np.frombuffer(f, dtype=np.uint8)
        poffs.append(pos)
        plens.append(len(f))
        pos += (len(f) + 15) & ~15
    del src
    stream = [prng.randrange(len(sizes)) for _ in range(nfiles)]
    gen_s = time.time() - t
    sbytes = sum(plens[i] for i in stream)
    # batches of consecutive stream files up to --batch-gib each (16-B aligned offsets)
    cap = int(a.batch_gib * (1 << 30))
    batches, cur, cpos = [], [], 0
    for fi in stream:
        ln = (plens[fi] + 15) & ~15
        if cur and cpos + ln > cap:
            batches.append(cur)
            cur, cpos = [], 0
        cur.append(fi)
        cpos += ln
    batches.append(cur)
    dev = torch.device("cuda", local)
    bufs = [torch.empty(cap + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
    ctx = W.Context(local)
    cs = torch.cuda.Stream(dev)
    copied = [torch.cuda.Event() for _ in range(2)]

    def enqueue(b):
        d = bufs[b % 2]
        offs, lens, o = [], [], 0
        with torch.cuda.stream(cs):
            for fi in batches[b]:
                d[o:o + plens[fi]].copy_(pool[poffs[fi]:poffs[fi] + plens[fi]], non_blocking=True)
                offs.append(o)
                lens.append(plens[fi])
                o += (plens[fi] + 15) & ~15
            copied[b % 2].record(cs)
        return offs, lens, o

    stt_all, kms, dms = [], [], []

    def run_all():
        stt_all.clear(), kms.clear(), dms.clear()
        nxt = enqueue(0)
        for b in range(len(batches)):
            offs, lens, used = nxt
            if b + 1 < len(batches):
                copied[b % 2].synchronize()        # batch b landed; (b+1)'s buffer is free
                nxt = enqueue(b + 1)
            else:
                copied[b % 2].synchronize()
            n = len(offs)
            st = (C.c_int32 * n)()
            rc = L.lib.esnap_verify_packed(ctx.handle, C.c_void_p(bufs[b % 2].data_ptr()), used,
                                           (C.c_uint64 * n)(*offs), (C.c_uint64 * n)(*lens), n, L.CASTAGNOLI, st,
                                           None, None)
            assert rc == 0, rc
            stt_all.extend(st)
            kms.append(float(L.lib.ewal_last_stream_ms(ctx.handle)))
            dms.append(float(L.lib.ewal_last_device_ms(ctx.handle)))

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_all()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    badset = set(pbad)
    want = [L.ERR_SNAP_CRC if fi in badset else L.OK for fi in stream]
    assert stt_all == want, "verdict mismatch"
    nbad = sum(1 for x in want if x != L.OK)
    used_total = sum(sum((plens[fi] + 15) & ~15 for fi in bt) for bt in batches)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # baseline only
        base_addr = pool.data_ptr()
        pick, acc = [], 0                 # a sample of the pool: the first files up to 2 GiB
        for i in range(len(plens)):
            if acc >= (2 << 30):
                break
            pick.append(i)
            acc += plens[i]
        so, sl = [poffs[i] for i in pick], [plens[i] for i in pick]
        small = [i for i in pick if plens[i] <= (8 << 20)][:64]
        views = [bytes(pv[poffs[i]:poffs[i] + plens[i]]) for i in small]
        vb = sum(len(v) for v in views)

        def one_pass():
            for v in views:
                O.loadsnap(v)
        csec = a.cpu_seconds if cpu_seconds is None else cpu_seconds
        it, cs = timed_cpu(csec, one_pass)
        nth = cpu_threads()
        it2, cs2 = timed_cpu(csec / 2, lambda: O.fast_snap_verify_batch(base_addr, so, sl, nth))
        cpu = dict(host_info(), **{
            "value": round(vb * it / cs / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle/ or_loadsnap (1 thread) over %d of the pool's files (<= 8 MiB each, %.2f GiB), %d "
                      "passes, %.1f s -- host-resident bytes, no PCIe" % (len(views), vb / (1 << 30), it, cs),
            "optimised": {"value": round(acc * it2 / cs2 / 1e9, 4), "unit": "GB/s", "cores": nth,
                          "sample": "orf_snap_verify_batch on %d cores over the pool's first %d files (%.2f GiB, "
                                    "pinned host memory), %d passes, %.1f s" % (nth, len(pick), acc / (1 << 30),
                                                                              it2, cs2)}})
    out = ({
            "metric": METRIC, "value": round(world * sbytes / el / 1e9, 3), "unit": "GB/s", "n_gpus": world,
            "steps": 1, "warmup": 0, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "configs[3] streamed: %d snapshot files (%.1f GiB) per GPU, sizes log-uniform "
                                   "1-256 MiB, drawn from a pinned pool of %d distinct files (%.1f GiB), %d corrupt "
                                   "in the stream; %d HBM batches of <= %.0f GiB, copies of batch b+1 overlapping "
                                   "the verification of batch b" % (nfiles, sbytes / (1 << 30), len(sizes),
                                                                    pos / (1 << 30), nbad, len(batches), a.batch_gib),
                       "files_per_gpu": nfiles, "snapshot_bytes_per_gpu": sbytes,
                       "parallelism": "dp%d (independent files)" % world},
            "files_per_s": round(world * nfiles / el, 1),
            "streamed_gbps_pinned": round(sbytes / el / 1e9, 3),
            "resident_gbps": round(used_total / (sum(dms) / 1e3) / 1e9, 2),
            "roofline": {"bound": "hbm", "achieved": round(used_total / (sum(kms) / 1e3) / 1e9, 2),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(used_total / (sum(kms) / 1e3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                         "kernel": "k_stream<false>", "kernel_ms": round(sum(kms) / len(kms), 4),
                         "algorithmic_bytes_per_launch": round(used_total / len(batches)),
                         "pipeline_achieved": round(used_total / (sum(dms) / 1e3) / 1e9, 2),
                         "pipeline_frac": round(used_total / (sum(dms) / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "note": "streamed value is PCIe-bound (host -> HBM); the roofline is the resident kernel"},
            "cpu_baseline": cpu, "gen_seconds": round(gen_s, 2)})
    ctx.close()
    return out


def run_restart(a, dist, rank, world, local):
    """The restart drop-in end to end: the configs[1]-
    shaped WAL (clean, 8 GiB) written as a WAL directory (tmpfs), then the
    cgo shim's call sequence as a C program (tests/shim/readall_shim.c):
    ctx create, OpenAtIndex (select + read the files), ewal_ctx_reserve, ReadAll
    (host -> HBM copy + the pipeline), the Go sentinel switch and the
    zero-copy materialisation of ~0.9 M raftpb.Entry -- each step timed.
    value = WAL GB/s over the whole restart."""
    import shutil
    import subprocess
    import tempfile
    size = int(a.size_gib * (1 << 30))
    buf, n = W.synth_wal(size, a.min_data, a.max_data, seed=2 + rank)
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    d = tempfile.mkdtemp(prefix="ewal_restart_", dir=base)
    try:
        with open(os.path.join(d, W.walName(0, 0)), "wb") as f:
            f.write(buf)
        nb = len(buf)
        del buf
        shim = os.path.join(ROOT, "tests", "shim", "readall_shim")
        runs = []
        for _ in range(max(1, a.steps)):
            p = subprocess.run([shim, d, "1"], capture_output=True, text=True, timeout=300)
            assert p.returncode == 0, p.stderr[-2000:]
            g = json.loads(p.stdout.strip().splitlines()[-1])
            assert g["sentinel"] == "nil" and g["n_records"] == n, g
            runs.append(g)
        cpu = None
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            # the same restart on the CPU, file read included (page cache / tmpfs, like the shim's)
            from oracle import oracle as O   # baseline only
            path = os.path.join(d, W.walName(0, 0))
            nth = cpu_threads()
            st, fr, rms, tms = O.restart_file(path, 1, 1, True)
            assert st == O.OK and fr == n, (st, fr, n)
            fast = []
            for _ in range(3):
                st2, fr2, rms2, tms2 = O.restart_file(path, 1, nth, False)
                assert st2 == O.OK and fr2 == n
                fast.append((tms2, rms2))
            tms2, rms2 = sorted(fast)[1]
            cpu = dict(host_info(), **{
                "value": round(nb / (tms / 1e3) / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
                "sample": "the whole restart: the %.2f GiB WAL file read (pread, 1 thread, %.0f ms) + oracle/ or_readall "
                          "(the faithful C restatement of wal.ReadAll, 1 thread), %.0f ms in all" % (nb / (1 << 30), rms, tms),
                "optimised": {"value": round(nb / (tms2 / 1e3) / 1e9, 4), "unit": "GB/s", "cores": nth,
                              "sample": "the file read by %d pread threads (%.0f ms) + orf_readall on %d cores "
                                        "(oracle/ewal_cpu_fast.c), %.0f ms in all (median of 3)" % (nth, rms2, nth, tms2)}})
    finally:
        shutil.rmtree(d, ignore_errors=True)
    best = min(runs, key=lambda g: g["ms"]["total"])
    med = sorted(runs, key=lambda g: g["ms"]["total"])[len(runs) // 2]
    out = ({
            "metric": METRIC, "value": round(world * nb / (med["ms"]["total"] / 1e3) / 1e9, 3), "unit": "GB/s",
            "n_gpus": world, "steps": len(runs), "warmup": 0, "ms_per_step": round(med["ms"]["total"], 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "restart: OpenAtIndex(dir, 1).ReadAll() through the C ABI as the cgo shim calls "
                                   "it, one %.2f GiB WAL file in tmpfs (configs[1] sizes, clean), %d frames, "
                                   "%d entries materialised as zero-copy views; a fresh process per restart"
                                   % (nb / (1 << 30), n, med["n_ents"]),
                       "wal_bytes": nb, "parallelism": "dp%d" % world},
            "steps_ms_median": med["ms"], "steps_ms_best": best["ms"], "device_ms": med["device_ms"],
            "readall_plus_materialise_ms": round(med["ms"]["readall"] + med["ms"]["materialise"], 3),
            "floor_note": "a fresh process pays the HIP runtime init (ctx_create, overlapped with the file reads "
                          "here) before any byte can cross PCIe; the rest is bounded by the host -> HBM copy of the "
                          "WAL bytes (~55 GB/s)",
            "cpu_baseline": cpu})
    return out


def run_commit(a, dist, rank, world, local, cpu_seconds=None):
    """configs[4]: batched raft.maybeCommit (raft/raft.go:248-258 +
    raft/log.go:148-154) over 1M raft groups per GPU, 5 or 7 voters (seed 6),
    a 16-entry log-term window per group.  The line times
    ecommit_batch_rec_device over 192-B group records (the voters' Match,
    committed, Term, log bounds and the log's last 13 terms: coalesced
    loads, no term gather for quorum indexes in that tail); `soa` times
    ecommit_batch_device over the SoA arrays (committed reset from a copy
    each step, so every step does the same work)."""
    import numpy as np
    G = 1 << 20
    rng = np.random.default_rng(6 + rank)
    nv = np.where(rng.random(G) < 0.5, 5, 7).astype(np.uint8)
    committed0 = rng.integers(0, 1 << 20, size=G, dtype=np.uint64)
    match = (committed0[None, :] + rng.integers(0, 24, size=(7, G), dtype=np.uint64)
             - np.uint64(4)).astype(np.uint64)
    term = rng.integers(1, 4, size=G, dtype=np.uint64)
    log_offset = committed0 + np.uint64(1) - rng.integers(0, 3, size=G, dtype=np.uint64)
    log_ptr = (np.arange(G + 1, dtype=np.uint64) * np.uint64(16))
    log_terms = np.sort(rng.integers(1, 4, size=(G, 16), dtype=np.uint64), axis=1).reshape(-1)
    dev = torch.device("cuda", local)
    T = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)   # noqa: E731
    d_match, d_nv, d_term, d_c0 = T(match.reshape(-1)), T(nv), T(term), T(committed0)
    d_off, d_ptr, d_lt = T(log_offset), T(log_ptr), T(log_terms)
    d_c = d_c0.clone()
    d_ch = torch.zeros(G, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(G, dtype=torch.uint8, device=dev)
    ctx = W.Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    cpu_seconds = a.cpu_seconds if cpu_seconds is None else cpu_seconds
    summary = torch.zeros(3, dtype=torch.int64, device=dev) if dist is not None else None
    dms = C.c_double(0)
    kms = []

    def step():
        d_c.copy_(d_c0)
        rc = L.lib.ecommit_batch_device(ctx.handle, G, C.c_void_p(d_match.data_ptr()), C.c_void_p(d_nv.data_ptr()),
                                        C.c_void_p(d_term.data_ptr()), C.c_void_p(d_c.data_ptr()),
                                        C.c_void_p(d_off.data_ptr()), C.c_void_p(d_ptr.data_ptr()),
                                        C.c_void_p(d_lt.data_ptr()), C.c_void_p(d_ch.data_ptr()),
                                        C.c_void_p(d_st.data_ptr()), C.byref(dms))
        assert rc == 0, rc
        kms.append(dms.value)
        if dist is not None:   # the node's commit-index summary (etcd_amd/shard.py), device scalars
            shard.combine_commit(dist, d_ch.sum(dtype=torch.int64), d_c.min(), d_c.max(), out=summary)

    for _ in range(max(a.warmup, 1)):
        step()
    new = d_c.cpu().numpy().view(np.uint64)
    ch = d_ch.cpu().numpy()
    assert (new >= committed0).all() and ((new != committed0) == (ch == 1)).all() and not d_st.cpu().numpy().any()
    nchanged = int(ch.sum())
    kms.clear()
    elapsed = timed(dist, a.steps, step)
    ms = elapsed / a.steps * 1e3
    k_avg = sum(kms) / len(kms)
    # algorithmic bytes: nvoters 1 + n match words + term, committed (r+w), log_offset, 2 log_ptr, the term gather,
    # changed + status
    abytes = int(G + 8 * int(nv.astype(np.int64).sum()) + G * (8 + 16 + 8 + 16 + 8 + 2))
    # ---- the same groups as 192-B records (ecommit_batch_rec_device) ----
    from etcd_amd import raftcommit as RC
    d_rec = T(RC.pack_groups(match, nv, committed0, term, log_offset, log_ptr, log_terms).reshape(-1))
    d_co = torch.zeros(G, dtype=torch.int64, device=dev)
    d_ch2 = torch.zeros(G, dtype=torch.uint8, device=dev)
    d_st2 = torch.zeros(G, dtype=torch.uint8, device=dev)
    P = lambda t: C.c_void_p(t.data_ptr())   # noqa: E731
    rkms = []

    def rstep(logs=True):
        rc = L.lib.ecommit_batch_rec_device(ctx.handle, G, P(d_rec), P(d_ptr) if logs else None,
                                            P(d_lt) if logs else None, P(d_co), P(d_ch2), P(d_st2), C.byref(dms))
        assert rc == 0, rc
        rkms.append(dms.value)
        if dist is not None:
            shard.combine_commit(dist, d_ch2.sum(dtype=torch.int64), d_co.min(), d_co.max(), out=summary)

    rstep(logs=False)   # (untimed) the groups whose quorum term lies before the tail window: they read the log
    n_gather = int((d_st2 == L.UNSUPPORTED_ENCODING).sum())
    for _ in range(max(a.warmup, 1)):
        rstep()
    bad = [int((d_co.cpu() != d_c.cpu()).sum()), int((d_ch2.cpu() != d_ch.cpu()).sum()),
           int((d_st2.cpu() != 0).sum())]
    assert bad == [0, 0, 0], "record path vs SoA path: committed / changed differ, status set: %s" % bad
    rkms.clear()
    rms = timed(dist, a.steps, rstep) / a.steps * 1e3
    rk_avg = sum(rkms) / len(rkms)
    # record 192 B + committed_out 8 + changed/status 2 per group; log_ptr + the term gather for n_gather groups
    rbytes = int(G * (192 + 8 + 2) + n_gather * 16)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # baseline only
        c = committed0.copy()
        chc, stc = np.zeros(G, np.uint8), np.zeros(G, np.uint8)
        it, t2 = 0, time.perf_counter()
        while True:
            c[:] = committed0
            O.maybe_commit_batch(G, match.reshape(-1), nv, term, c, log_offset, log_ptr, log_terms, chc, stc)
            it += 1
            if time.perf_counter() - t2 >= cpu_seconds:
                break
        cs = time.perf_counter() - t2
        nth = cpu_threads()

        def all_cores():
            c[:] = committed0
            O.fast_maybe_commit_batch(G, match.reshape(-1), nv, term, c, log_offset, log_ptr, log_terms, chc, stc, nth)
        it2, cs2 = timed_cpu(cpu_seconds / 2, all_cores)
        cpu = dict(host_info(), **{
            "value": round(G * it / cs, 1), "unit": "groups/s", "cores": 1, "kind": "port",
            "sample": "oracle/ or_maybe_commit_batch (insertion sort + q-th largest + term check per group, 1 "
                      "thread) over all %d groups, %d passes, %.1f s" % (G, it, cs),
            "optimised": {"value": round(G * it2 / cs2, 1), "unit": "groups/s", "cores": nth,
                          "sample": "the same per-group code on all %d cores over group ranges "
                                    "(orf_maybe_commit_batch), %d passes, %.1f s" % (nth, it2, cs2)}})
    out = {
            "metric": "maybeCommit groups/s (configs[4]); WAL verify GB/s is the headline metric",
            "value": round(world * G / (rms / 1e3), 1), "unit": "groups/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(rms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "configs[4]: maybeCommit over %d raft groups per GPU, 5/7 voters (50/50), 16-entry "
                                   "log-term window; %d groups advance commit; one ecommit_batch_rec_device per step "
                                   "(192-B group records, the log's last 13 terms inside; %d groups read their "
                                   "quorum term from the log arrays)" % (G, nchanged, n_gather),
                       "groups_per_gpu": G, "parallelism": "dp%d (group ranges)" % world},
            # algorithmic bytes: the SAME model as the soa line (the bytes maybeCommit needs per group: the
            # voters' Match, Term, committed r+w, the log bounds, the quorum term, changed + status), so the
            # two kernels' fractions compare like for like; the 192-B records the kernel actually streams
            # (unused voter slots and tail terms included) are reported as bytes_moved
            "roofline": {"bound": "hbm", "achieved": round(abytes / (rk_avg / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(abytes / (rk_avg / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "traffic": load_traffic("k_commit_rec"), "kernel": "k_commit_rec",
                         "kernel_ms": round(rk_avg, 4), "algorithmic_bytes_per_launch": abytes,
                         "bytes_moved_per_launch": rbytes,
                         "bytes_moved_gbps": round(rbytes / (rk_avg / 1e3) / 1e9, 2),
                         "traffic_source": "profiles/k_commit_rec_pmc.json: the committed rocprofv3 PMC pass of this "
                                           "config (FETCH_SIZE x2 + WRITE_SIZE per launch), not measured in this run",
                         "note": "raftcommit.pack_groups (host numpy, once before the loop) is not timed: the "
                                 "record layout is the caller's storage format, like the SoA arrays"},
            "soa": {"note": "the same groups through ecommit_batch_device (SoA match[v*G+g], log_terms gather; "
                            "committed reset from a copy each step)", "ms_per_step": round(ms, 4),
                    "value": round(world * G / (ms / 1e3), 1),
                    "roofline": {"bound": "hbm", "achieved": round(abytes / (k_avg / 1e3) / 1e9, 2),
                                 "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                 "frac": round(abytes / (k_avg / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                                 "traffic": load_traffic("k_commit"), "kernel": "k_commit",
                                 "kernel_ms": round(k_avg, 4), "algorithmic_bytes_per_launch": abytes,
                                 "traffic_source": "profiles/k_commit_pmc.json (the 8-B term gather costs a whole "
                                                   "128-B line per group)"}},
            "cpu_baseline": cpu}
    ctx.close()
    return out


def run_msg(a, dist, rank, world, local):
    """batched raftpb.Message decode for the /raft
    ingress (raft/raftpb/raft.pb.go:407-617): 256 Ki message bodies resident
    in HBM (1024 distinct bodies tiled: MsgApp with 1-8 entries of 64 B-1 KiB,
    heartbeats and votes with none), one emsg_decode_batch_device per step
    (count pass, scan, decode pass, results copied to the host)."""
    import random
    from etcd_amd import raftmsg as M
    rng = random.Random(9 + rank)
    distinct, nents = [], []
    for i in range(1024):
        ne = rng.choice([0, 0, 1, 2, 4, 8])
        nents.append(ne)
        ents = [M.entry_marshal(0, 5, 1000 + i * 8 + k, rng.randbytes(rng.randrange(64, 1025))) for k in range(ne)]
        distinct.append(M.message_marshal(3 if ne else rng.choice([1, 5, 8]), 2, 1, 5, 5, 1000 + i * 8, ents,
                                          999 + i, b"", False))
    n = 256 * 1024
    bodies = [distinct[i % len(distinct)] for i in range(n)]
    lens = [len(b) for b in bodies]
    offs, pos = [], 0
    for x in lens:
        offs.append(pos)
        pos += x
    blob = b"".join(bodies)
    nb = len(blob)
    ctx = W.Context(local)
    dbuf = ctx.alloc(nb + 64)
    dbuf.upload(blob)
    co, cl = (C.c_uint64 * n)(*offs), (C.c_uint64 * n)(*lens)
    out = (L.MessageDesc * n)()
    tot = C.c_uint64(0)

    def step():
        rc = L.lib.emsg_decode_batch_device(ctx.handle, dbuf.ptr, nb, co, cl, n, out, C.byref(tot))
        assert rc == 0, rc

    for _ in range(max(a.warmup, 1)):
        step()
    want_ents = sum(nents[i % len(distinct)] for i in range(n))
    assert all(m.status == 0 for m in out) and tot.value == want_ents, (tot.value, want_ents)
    elapsed = timed(dist, a.steps, step)
    ms = elapsed / a.steps * 1e3
    dms = float(L.lib.ewal_last_device_ms(ctx.handle))
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # baseline only
        addr = C.cast(C.c_char_p(blob), C.c_void_p).value
        stc = O.fast_message_batch(addr, offs, lens, 1)
        assert all(x == O.OK for x in stc)
        it, cs = timed_cpu(a.cpu_seconds, lambda: O.fast_message_batch(addr, offs, lens, 1))
        nth = cpu_threads()
        it2, cs2 = timed_cpu(a.cpu_seconds / 2, lambda: O.fast_message_batch(addr, offs, lens, nth))
        cpu = dict(host_info(), **{
            "value": round(n * it / cs, 1), "unit": "messages/s", "cores": 1, "kind": "port",
            "sample": "oracle/ or_message_unmarshal (the C restatement of raftpb.Message.Unmarshal, a fresh message "
                      "per body) over all %d bodies, 1 thread, %d passes, %.1f s" % (n, it, cs),
            "optimised": {"value": round(n * it2 / cs2, 1), "unit": "messages/s", "cores": nth,
                          "sample": "the same per message on %d cores, %d passes, %.1f s" % (nth, it2, cs2)}})
    out = ({
            "metric": "raftpb.Message decode messages/s (SURVEY 8(f) rank 4); WAL verify GB/s is the headline",
            "value": round(world * n / (ms / 1e3), 1), "unit": "messages/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "%d raftpb.Message bodies (%.1f MB) per GPU, %d entries decoded per step; "
                                   "results copied to the host each step" % (n, nb / 1e6, tot.value),
                       "parallelism": "dp%d" % world},
            "gbps": round(world * nb / (ms / 1e3) / 1e9, 3), "device_ms": round(dms, 4),
            "cpu_baseline": cpu})
    dbuf.free()
    ctx.close()
    return out


def run_wal(a, dist, rank, world, local, size, min_data, max_data, label, cpu_seconds, full=True):
    """configs[1] (and configs[0]'s WAL as `c1`): one ReadAll per step over a
    GPU-resident WAL per rank with one corrupt record at frame 0.73 N.  full:
    the headline's extras -- the clean WAL timed in the loop too, first-call
    and PCIe-inclusive (host -> HBM) rates."""
    buf_t = time.time()
    buf, n = W.synth_wal(size, min_data, max_data, seed=2 + rank)
    nb = len(buf)
    gen_s = time.time() - buf_t
    ctx = W.Context(local)
    dbuf = ctx.alloc(nb + 64)
    dbuf.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
    extra = {}
    if full:
        # the one-shot restart (etcdserver/server.go:153-156) in a cold process: ewal_ctx_reserve first (device
        # code load + workspace; a server runs it while it reads the WAL files), then the first ReadAll
        tf = time.perf_counter()
        rc0 = L.lib.ewal_ctx_reserve(ctx.handle, nb, 0)
        extra["reserve_ms_cold"] = round((time.perf_counter() - tf) * 1e3, 3)
        assert rc0 == 0, rc0
        tf = time.perf_counter()
        r = W.readall_device(dbuf, nb, 1)
        extra["first_call_reserved_ms"] = round((time.perf_counter() - tf) * 1e3, 3)
        assert r.status == L.OK and r.n_records == n, (r.status, r.n_records, n)
        # ... and on a fresh ctx without the reserve (it sizes its workspace itself; device code already loaded)
        ctx2 = W.Context(local)
        r2 = L.Result()
        tf = time.perf_counter()
        L.lib.ewal_readall_device(ctx2.handle, dbuf.ptr, nb, 1, C.byref(r2))
        extra["first_call_ms"] = round((time.perf_counter() - tf) * 1e3, 3)
        assert r2.status == L.OK and r2.n_records == n
        ctx2.close()
        extra["first_call_note"] = ("reserve_ms_cold: ewal_ctx_reserve in a cold process (device code load + "
                                    "workspace), then first_call_reserved_ms; first_call_ms: a fresh ctx without "
                                    "the reserve")
    r = W.readall_device(dbuf, nb, 1)
    assert r.status == L.OK and r.n_records == n, (r.status, r.n_records, n)
    rs = L.Result()      # the C ABI straight into a preallocated result: no Python objects in the timed region
    if full:
        # the clean WAL (the common restart case: ents placed, the result gathered), timed in the loop
        def clean_step():
            rc = L.lib.ewal_readall_device(ctx.handle, dbuf.ptr, nb, 1, C.byref(rs))
            assert rc == L.OK and rs.n_records == n, (rc, rs.n_records)
        clean_step()
        extra["clean_ms_per_step"] = round(timed(dist, a.steps, clean_step) / a.steps * 1e3, 4)
        extra["clean_pipeline_device_ms"] = round(rs.device_ms, 4)
    k = int(0.73 * n)
    rec = W.records(ctx, n)[k]
    p = rec["data_off"] + rec["data_len"] // 2
    flip = bytearray(dbuf.download(1, p))
    flip[0] ^= 0x5A
    dbuf.upload(bytes(flip), p)
    buf[p] ^= 0x5A     # keep the host copy identical (E2E and CPU legs)

    # ---- warmup + correctness gate -----------------------------------------
    for _ in range(max(a.warmup, 1)):
        r = W.readall_device(dbuf, nb, 1)
    assert r.status == L.ERR_RECORD_CRC and r.fail_record == k, (r.status, r.fail_record, k)

    summary = torch.zeros(3, dtype=torch.int64, device="cuda") if dist is not None else None
    stream_ms, dev_ms, post_ms, fr_ms = [], [], [], []

    def step():
        rc = L.lib.ewal_readall_device(ctx.handle, dbuf.ptr, nb, 1, C.byref(rs))
        assert rc == L.ERR_RECORD_CRC and rs.fail_record == k, (rc, rs.fail_record)
        stream_ms.append(rs.stream_ms)
        dev_ms.append(rs.device_ms)
        post_ms.append(rs.post_ms)
        fr_ms.append(rs.frames_ms)
        if dist is not None:   # one all-reduce of the shard verdicts (etcd_amd/shard.py)
            shard.combine(dist, rank, rs.fail_record, rs.n_records, rs.status != L.OK, out=summary)

    elapsed = timed(dist, a.steps, step)
    ms_per_step = elapsed / a.steps * 1e3
    gbps = world * nb / (ms_per_step / 1e3) / 1e9
    recs_per_s = world * n / (ms_per_step / 1e3)
    stream_avg = sum(stream_ms) / len(stream_ms)
    dev_avg = sum(dev_ms) / len(dev_ms)
    post_avg = sum(post_ms) / len(post_ms)
    fr_avg = sum(fr_ms) / len(fr_ms)
    achieved = nb / (stream_avg / 1e3) / 1e9

    # ---- end-to-end variant (host -> device included), one pass -------------
    if full and not a.no_e2e:
        t1 = time.perf_counter()
        rr = L.Result()
        bptr = C.addressof((C.c_char * nb).from_buffer(buf))
        rc = L.lib.ewal_readall_host(ctx.handle, C.c_void_p(bptr), nb, 1, C.byref(rr))
        e2e_s = time.perf_counter() - t1
        assert rc == L.ERR_RECORD_CRC and rr.fail_record == k
        extra["e2e_gbps_incl_h2d"] = round(nb / e2e_s / 1e9, 3)

    # ---- CPU baseline: oracle ReadAll (Go-faithful port) on a bounded sample -
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # checker / baseline only
        # the sample: the frames before the first one at or past 1 GiB (or before the corrupt one)
        r = W.readall_device(dbuf, nb, 1)
        cutr = W.records(ctx, k)
        cut = next((x["offset"] for x in cutr if x["offset"] >= (1 << 30)), cutr[-1]["offset"])
        sample = bytes(buf[:cut])
        iters, t2 = 0, time.perf_counter()
        while True:
            o = O.readall(sample, 1)
            iters += 1
            if time.perf_counter() - t2 >= cpu_seconds:
                break
        cpu_s = time.perf_counter() - t2
        assert o["status"] == O.OK
        # the optimised CPU ReadAll on the CPU share, over the whole WAL (its corrupt frame included)
        nth = cpu_threads()
        addr = C.addressof((C.c_char * nb).from_buffer(buf))
        fst = O.fast_readall_status(addr, nb, 1, nth)
        assert fst[0] == O.ERR_RECORD_CRC and fst[2] == k, fst
        it2, cs2 = timed_cpu(cpu_seconds / 2, lambda: O.fast_readall_status(addr, nb, 1, nth))
        it3, cs3 = timed_cpu(cpu_seconds / 4, lambda: O.fast_readall_status(addr, nb, 1, 1))
        cpu = dict(host_info(), **{
            "value": round(len(sample) * iters / cpu_s / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle/ or_readall (C restatement of wal.ReadAll: per-record alloc+copy, SSE4.2 "
                      "CRC-32C, 1 thread) over the first %.2f GiB (%d frames) of the same WAL, %d passes, "
                      "%.1f s" % (len(sample) / (1 << 30), o["n_records"], iters, cpu_s),
            "optimised": {"value": round(nb * it2 / cs2 / 1e9, 4), "unit": "GB/s", "cores": nth,
                          "one_core_gbps": round(nb * it3 / cs3 / 1e9, 4),
                          "sample": "oracle/ewal_cpu_fast.c orf_readall over the whole %.2f GiB WAL (stops at the "
                                    "corrupt frame %d like the reference): serial framing walk, every frame's CRC "
                                    "with the local-verify rule on %d cores (3-stream SSE4.2 CRC-32C), ReadAll's "
                                    "dispatch over the frame table; %d passes, %.1f s" %
                                    (nb / (1 << 30), k, nth, it2, cs2)}})
    out = {
        "metric": METRIC, "value": round(gbps, 3), "unit": "GB/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "%s: one %.3f GiB WAL per GPU, %d frames, entry Data log-uniform "
                               "%d B-%d B, 1 corrupt record at frame %d (walpb.ErrCRCMismatch)"
                               % (label, nb / (1 << 30), n, min_data, max_data, k),
                   "wal_bytes_per_gpu": nb, "frames_per_gpu": n, "ri": 1,
                   "parallelism": "dp%d (independent WAL shards)" % world},
        "records_per_s": round(recs_per_s, 1),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": load_traffic() if label == "configs[1]" else None,
                     "kernel": "k_stream", "kernel_ms": round(stream_avg, 4),
                     "algorithmic_bytes_per_launch": nb,
                     "pipeline_achieved": round(nb / (dev_avg / 1e3) / 1e9, 2),
                     "pipeline_frac": round(nb / (dev_avg / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "step_frac": round(gbps / world / HBM_PEAK_GBPS, 4)},
        "pipeline_device_ms": round(dev_avg, 4),
        "post_stream_ms": round(post_avg, 4),
    }
    if fr_avg:   # the frame pass ran as one launch after the stream pass: its own roofline entry
        wk = "wal" if label == "configs[1]" else ("c1" if label.startswith("configs[0]") else "none")
        out["roofline_frames"] = frames_roofline(n, nb, fr_avg, wk)
        if fr_avg > stream_avg:   # the dominant kernel by time names the line's roofline
            out["roofline"], out["roofline_stream"] = out["roofline_frames"], out["roofline"]
            del out["roofline_frames"]
    else:
        out["pipeline"] = ("overlapped: the stream pass in chunks on %s CUs, each chunk's frame pass on the other CUs "
                           "as it completes; post_stream_ms = the part after the last stream chunk" %
                           "most")
    if label == "configs[1]":
        out["roofline"]["traffic_source"] = ("profiles/k_stream_pmc.json: the committed rocprofv3 PMC pass of this "
                                             "config (FETCH_SIZE x2 + WRITE_SIZE per launch), not measured in this run")
    out.update(extra)
    out["cpu_baseline"] = cpu
    out["gen_seconds"] = round(gen_s, 2)
    dbuf.free()
    ctx.close()
    del buf
    return out


def run_rewind(a, dist, rank, world, local, cpu_seconds=None):
    """A configs[1]-shaped WAL (8 GiB, 64 B - 64 KiB entries) after leader
    changes: 1 % of the entries open a new leader's term that rewrites the
    last 1..8 indexes (wal/wal.go:170-176, ents = append(ents[:Index-ri], e)),
    clean otherwise -- the irregular input a restart after an election sees.
    One ReadAll per step; every step returns len(ents) == the last Index."""
    cpu_seconds = a.cpu_seconds if cpu_seconds is None else cpu_seconds
    t = time.time()
    li = []
    buf, n = W.synth_wal(8 << 30, 64, 65536, seed=22 + rank, rewind_per_mille=10, last_index=li)
    nb = len(buf)
    gen_s = time.time() - t
    ctx = W.Context(local)
    dbuf = ctx.alloc(nb + 64)
    dbuf.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
    rs = L.Result()

    def step():
        rc = L.lib.ewal_readall_device(ctx.handle, dbuf.ptr, nb, 1, C.byref(rs))
        assert rc == L.OK and rs.n_records == n and rs.n_ents == li[0], (rc, rs.n_records, rs.n_ents, li[0])

    for _ in range(max(a.warmup, 1)):
        step()
    ms = timed(dist, a.steps, step) / a.steps * 1e3
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # baseline only
        cut = 1 << 30
        p, last = 0, 0
        while p + 8 <= nb and p < cut:      # the frames in the first GiB (length prefixes)
            last = p
            p += 8 + int.from_bytes(buf[p:p + 8], "little")
        sample = bytes(buf[:p if p <= nb else last])
        it, cs = timed_cpu(cpu_seconds, lambda: O.readall(sample, 1))
        o = O.readall(sample, 1)
        assert o["status"] == O.OK
        cpu = dict(host_info(), **{
            "value": round(len(sample) * it / cs / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle/ or_readall (the faithful C restatement of wal.ReadAll, 1 thread) over the first "
                      "%.2f GiB (%d frames) of the same WAL, %d passes, %.1f s" % (len(sample) / (1 << 30),
                                                                                  o["n_records"], it, cs)})
    out = {
        "metric": METRIC, "value": round(world * nb / (ms / 1e3) / 1e9, 3), "unit": "GB/s",
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4), "dtype": "u8",
        "config": {"workload": "configs[1]-shaped WAL after leader changes: %.3f GiB, %d frames, 1 %% of the entries "
                               "rewrite the last 1-8 indexes (new term); clean, one ReadAll per step -> %d ents"
                               % (nb / (1 << 30), n, li[0]),
                   "wal_bytes_per_gpu": nb, "frames_per_gpu": n, "ri": 1},
        "records_per_s": round(world * n / (ms / 1e3), 1),
        "roofline": {"bound": "hbm", "achieved": round(nb / (rs.stream_ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(nb / (rs.stream_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "traffic": None, "kernel": "k_stream", "kernel_ms": round(rs.stream_ms, 4),
                     "algorithmic_bytes_per_launch": nb,
                     "pipeline_achieved": round(nb / (rs.device_ms / 1e3) / 1e9, 2),
                     "pipeline_frac": round(nb / (rs.device_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "step_frac": round(nb / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "pipeline_device_ms": round(rs.device_ms, 4),
        "cpu_baseline": cpu, "gen_seconds": round(gen_s, 2)}
    dbuf.free()
    ctx.close()
    del buf
    return out


def run_split(a, dist, rank, world, local, cpu_seconds=None, nctx=2):
    """configs[1]'s WAL read as ONE WAL split over `nctx` contexts on THIS
    GPU (ewal_multi_readall_device: the ranges stay where they lie in HBM,
    each opening at a 16-B aligned frame start; one host thread per ctx; the
    verdict, metadata, HardState and len(ents) joined in C).  A one-GPU
    rehearsal of the multi-GPU split of SURVEY §8(e) -- both ranges share one
    GPU's CUs and HBM, so this is not scaling data.  Checked against the
    single-ctx ReadAll of the same bytes before the timed steps."""
    buf, n = W.synth_wal(int(a.size_gib * (1 << 30)), a.min_data, a.max_data, seed=2 + rank)
    nb = len(buf)
    ctxs = [W.Context(local) for _ in range(nctx)]
    d = ctxs[0].alloc(nb + 64)
    d.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
    one = W.readall_device(d, nb, 1, host_view=memoryview(buf))   # (the metadata bytes from the host copy)
    assert one.status == L.OK and one.n_records == n, (one.status, one.n_records)
    m = W.Multi(ctxs)
    t0 = time.perf_counter()
    plan = m.plan_device(d, nb, 1)
    plan_ms = (time.perf_counter() - t0) * 1e3
    g = m.readall_device(d, nb, 1, plan=plan)
    assert (g.status, g.n_records, g.last_crc, g.enti, g.metadata, g.state) == \
        (one.status, one.n_records, one.last_crc, one.enti, one.metadata, one.state), (g.status, g.n_records)
    assert m.timing()["resplits"] == 0
    tim = []

    def step():
        r = m.readall_device(d, nb, 1, plan=plan)
        assert r.status == L.OK and r.n_records == n, (r.status, r.n_records)
        tim.append(m.timing())

    for _ in range(max(a.warmup, 1)):
        step()
    tim.clear()
    ms = timed(dist, a.steps, step) / a.steps * 1e3
    avg = lambda k: sum(t[k] for t in tim) / len(tim)   # noqa: E731
    out = {"metric": METRIC, "value": round(world * nb / (ms / 1e3) / 1e9, 3), "unit": "GB/s",
           "ms_per_step": round(ms, 4), "steps": a.steps, "dtype": "u8",
           "config": {"workload": "configs[1]'s %.2f GiB WAL as ONE WAL split over %d contexts on one GPU "
                                  "(device-resident ranges at %s)" % (nb / (1 << 30), nctx, plan[0]),
                      "wal_bytes": nb, "frames": n, "ranges": nctx, "parallelism": "one-GPU rehearsal"},
           "range_device_ms_max": round(avg("max_range_device_ms"), 4),
           "join_host_ms": round(avg("join_ms"), 4), "call_wall_ms": round(avg("wall_ms"), 4),
           "plan_ms": round(plan_ms, 3), "resplits": int(avg("resplits")),
           "note": "rehearsal, not scaling data: the ranges share one GPU; each range's ReadAll is followed by "
                   "ewal_copy_range_info (read from the frame pass's reductions, k_range_info_fr) for the join"}
    m.close()
    d.free()
    for c in ctxs:
        c.close()
    return out


SUBS = {"c1": None, "shards": run_shards, "snap": run_snap, "snapstream": run_snapstream, "commit": run_commit,
        "rewind": run_rewind, "split2": run_split}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = 0 if a.one_device else int(os.environ.get("LOCAL_RANK", "0"))

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(a.dist_backend)

    c1 = dict(size=int(285e6), min_data=256, max_data=256, label="configs[0] WAL on the GPU")
    failed = []   # sub-configs that raised (their parity / gate asserts included): the run exits non-zero
    if a.workload in ("wal", "c1"):
        if a.workload == "c1":
            out = run_wal(a, dist, rank, world, local, cpu_seconds=a.cpu_seconds, full=False, **c1)
        else:
            label = "configs[1]" if (a.size_gib, a.min_data, a.max_data) == (8.0, 64, 65536) else "configs[1]-shaped"
            out = run_wal(a, dist, rank, world, local, int(a.size_gib * (1 << 30)), a.min_data, a.max_data, label,
                          a.cpu_seconds)
            subs = [x for x in a.configs.split(",") if x and x != "none"] if a.workload == "wal" else []
            if subs:
                out["configs"] = {}
            for name in subs:
                t0 = time.time()
                try:
                    if name == "c1":
                        r = run_wal(a, dist, rank, world, local, cpu_seconds=a.sub_cpu_seconds, full=False, **c1)
                    else:
                        r = SUBS[name](a, dist, rank, world, local, cpu_seconds=a.sub_cpu_seconds)
                except Exception as ex:   # the headline line still prints, the failure is in it, and rc != 0
                    import traceback
                    traceback.print_exc()
                    r = {"error": "%s: %s" % (type(ex).__name__, ex), "ms_per_step": None}
                    failed.append(name)
                r["wall_seconds"] = round(time.time() - t0, 2)
                for key in ("higher_is_better", "scaling", "vs_baseline", "data", "n_gpus"):
                    r.pop(key, None)
                out["configs"][name] = r
                if rank == 0:
                    print("bench: %s %s ms/step (%.1f s)" % (name, r["ms_per_step"], r["wall_seconds"]),
                          file=sys.stderr, flush=True)
    else:
        out = {"shards": run_shards, "snap": run_snap, "snapstream": run_snapstream, "commit": run_commit,
               "msg": run_msg, "restart": run_restart, "rewind": run_rewind}[a.workload](a, dist, rank, world, local)
    if rank == 0:
        import resource   # this rank's peak host memory (synthetic inputs, pinned snapshot pool): for N-rank nodes
        out["host_peak_rss_gib"] = round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / (1 << 20), 2)
        if failed:
            out["failed_configs"] = failed
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if failed:
        print("bench: FAILED sub-configs: %s" % ",".join(failed), file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
