#!/usr/bin/env python3
"""bench.py -- etcd WAL replay-and-verify on MI355X (BASELINE.json metric).

One step = one (*WAL).ReadAll (wal/wal.go:164-216) over a GPU-resident
synthetic WAL of configs[1]: 8 GiB of mixed 64 B - 64 KiB entries
(log-uniform sizes, xorshift payload) with one corrupt record at frame
k = 0.73 N, so every step must report walpb.ErrCRCMismatch at frame k.
The whole WAL is read and verified each step (the GPU pipeline does not
stop early).  With --gpus N (torchrun), every rank verifies its own
independent WAL shard (weak scaling) and one RCCL all-reduce per step
combines {MIN first-corrupt key, SUM frames, SUM mismatches}.

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
    return ap.parse_args()


def load_traffic():
    """Per-launch HBM bytes of k_stream from the committed PMC pass, if any."""
    p = os.path.join(ROOT, "profiles", "k_stream_pmc.json")
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    def barrier():
        if dist is not None:
            dist.barrier()

    # ---- input: an independent synthetic WAL shard per rank ----------------
    size = int(a.size_gib * (1 << 30))
    t = time.time()
    buf, n = W.synth_wal(size, a.min_data, a.max_data, seed=2 + rank)
    nb = len(buf)
    gen_s = time.time() - t
    ctx = W.Context(local)
    dbuf = ctx.alloc(nb + 64)
    dbuf.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
    r = W.readall_device(dbuf, nb, 1)
    assert r.status == L.OK and r.n_records == n, (r.status, r.n_records, n)
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

    summary = None
    if dist is not None:
        summary = torch.zeros(3, dtype=torch.int64, device="cuda")

    # ---- timed region --------------------------------------------------------
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stream_ms, dev_ms = [], []
    for _ in range(a.steps):
        r = W.readall_device(dbuf, nb, 1)
        stream_ms.append(r.stream_ms)
        dev_ms.append(r.device_ms)
        if dist is not None:   # one all-reduce of the shard verdicts (etcd_amd/shard.py)
            shard.combine(dist, rank, r.fail_record, r.n_records, r.status != L.OK, out=summary)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / a.steps * 1e3
    gbps = world * nb / (ms_per_step / 1e3) / 1e9
    recs_per_s = world * n / (ms_per_step / 1e3)

    stream_avg = sum(stream_ms) / len(stream_ms)
    achieved = nb / (stream_avg / 1e3) / 1e9

    # ---- end-to-end variant (host -> device included), one pass -------------
    e2e = None
    if not a.no_e2e:
        t1 = time.perf_counter()
        rr = L.Result()
        bptr = C.addressof((C.c_char * nb).from_buffer(buf))
        rc = L.lib.ewal_readall_host(ctx.handle, C.c_void_p(bptr), nb, 1, C.byref(rr))
        e2e_s = time.perf_counter() - t1
        assert rc == L.ERR_RECORD_CRC and rr.fail_record == k
        e2e = round(nb / e2e_s / 1e9, 3)

    # ---- CPU baseline: oracle ReadAll (Go-faithful port) on a bounded sample -
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O   # checker / baseline only
        recs = W.records(ctx, k)         # frames before the corrupt one
        cut = next((x["offset"] for x in recs if x["offset"] >= (1 << 30)), recs[-1]["offset"])
        sample = bytes(buf[:cut])
        iters, t2 = 0, time.perf_counter()
        while True:
            o = O.readall(sample, 1)
            iters += 1
            if time.perf_counter() - t2 >= a.cpu_seconds:
                break
        cpu_s = time.perf_counter() - t2
        assert o["status"] == O.OK
        cpu = {"value": round(len(sample) * iters / cpu_s / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
               "sample": "oracle/ or_readall (C restatement of wal.ReadAll: per-record alloc+copy, SSE4.2 "
                         "CRC-32C, 1 thread) over the first %.2f GiB (%d frames) of the same WAL, %d passes, "
                         "%.1f s" % (len(sample) / (1 << 30), o["n_records"], iters, cpu_s)}

    if rank == 0:
        out = {
            "metric": "WAL verify GB/s (and records/s) per GPU + 8-GPU node, % of HBM roofline",
            "value": round(gbps, 3), "unit": "GB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "configs[1]: one %.2f GiB WAL per GPU, %d frames, entry Data log-uniform "
                                   "%d B-%d KiB, 1 corrupt record at frame %d (walpb.ErrCRCMismatch)"
                                   % (nb / (1 << 30), n, a.min_data, a.max_data // 1024, k),
                       "wal_bytes_per_gpu": nb, "frames_per_gpu": n, "ri": 1,
                       "parallelism": "dp%d (independent WAL shards)" % world},
            "records_per_s": round(recs_per_s, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": load_traffic(),
                         "kernel": "k_stream", "kernel_ms": round(stream_avg, 4),
                         "algorithmic_bytes_per_launch": nb},
            "pipeline_device_ms": round(sum(dev_ms) / len(dev_ms), 4),
            "e2e_gbps_incl_h2d": e2e,
            "cpu_baseline": cpu,
            "gen_seconds": round(gen_s, 2),
        }
        print(json.dumps(out), flush=True)
    dbuf.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
