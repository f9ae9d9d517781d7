"""Per-phase cycles of k_frames (a -DFR_TIMING build of the library, loaded
through EWAL_LIB_PATH): the configs[1] WAL and configs[0]'s WAL on the GPU.
Usage: EWAL_LIB_PATH=tools/libewal_tm.so python tools/fr_timing.py [wal] [c1] [shards]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from etcd_amd import _lib as L
from etcd_amd import wal as W

NAMES = ["stage", "A", "pieces", "decode", "checks", "ops", "reduce", "tile_end"]
lib = L.lib
lib.ewal_dbg_fr_timing.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.ewal_dbg_fr_seam_timing.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.ewal_dbg_fr_seam_steps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.ewal_dbg_fr_wave_times.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.ewal_dbg_fr_seam_maxsteps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.ewal_dbg_fr_result_steps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]


def one(label, size, lo, hi, nsh=0):
    """nsh > 0: a configs[2]-shaped batch of nsh shards of `size` bytes each (one batched ReadAll)"""
    if nsh:
        buf, lens, nrec = W.synth_shards(list(range(nsh)), size, lo, hi)
        n = sum(nrec)
    else:
        buf, n = W.synth_wal(size, lo, hi, seed=2)
        lens = [len(buf)]
    ctx = W.Context(0)
    nb = len(buf)
    d = ctx.alloc(nb + 64)
    d.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
    rs = L.Result()
    mx = (C.c_ulonglong * (1024 * 8))()
    ns = len(lens)
    cl, cr, co = (C.c_uint64 * ns)(*lens), (C.c_uint64 * ns)(*([1] * ns)), (L.Result * ns)()
    for i in range(3):
        if i == 2:   # the per-block maxima accumulate: zeroed before the measured call
            lib.ewal_dbg_fr_seam_maxsteps(mx, 1024 * 8)
        if nsh:
            rc = lib.ewal_readall_batch_device(ctx.handle, d.ptr, ns, cl, cr, co)
            rs = co[0]
            assert rc == 0 and all(x.status == 0 and not (x.flags & L.FLAG_SHARD_FALLBACK) for x in co)
        else:
            rc = lib.ewal_readall_device(ctx.handle, d.ptr, nb, 1, C.byref(rs))
            assert rc == 0 and rs.flags & L.FLAG_FAST_PATH, (rc, rs.flags)
    t = (C.c_ulonglong * (8192 * 8))()
    lib.ewal_dbg_fr_timing(t, 8192 * 8)
    sd = (C.c_ulonglong * (1024 * 4))()
    lib.ewal_dbg_fr_seam_timing(sd, 1024 * 4)
    blocks = [list(sd[b * 4:(b + 1) * 4]) for b in range(1024) if sd[b * 4 + 2]]
    if blocks:
        t0 = min(b[2] for b in blocks)
        print("  seam: %d blocks, loop avg %.0f max %.0f cycles, last block ends loop at +%.0f, fr_result %.0f" %
              (len(blocks), sum(b[0] for b in blocks) / len(blocks), max(b[0] for b in blocks),
               max(b[3] for b in blocks) - t0, max(b[1] for b in blocks)))
    st = (C.c_ulonglong * (1024 * 8))()
    lib.ewal_dbg_fr_seam_steps(st, 1024 * 8)
    rows = [list(st[b * 8:(b + 1) * 8]) for b in range(1024) if any(st[b * 8:(b + 1) * 8])]
    if rows:
        print("  seam thread 0 steps (cycles from the loop start, median over blocks): " +
              " ".join("%s=%d" % (nm, sorted(r[i] for r in rows)[len(rows) // 2])
                       for i, nm in ((1, "loads"), (2, "first"), (3, "last"), (4, "end"), (5, "staging"),
                                     (6, "wait+fold"), (7, "atomics+fence"))) +
              "  (wait+fold includes this timing build's own 1024 same-line atomics per block)")
    lib.ewal_dbg_fr_seam_maxsteps(mx, 1024 * 8)
    rows = [list(mx[b * 8:(b + 1) * 8]) for b in range(1024) if any(mx[b * 8:(b + 1) * 8])]
    if rows:
        print("  seam slowest thread per block (cycles from the loop start; median / max over blocks): " +
              " ".join("%s=%d/%d" % (nm, sorted(r[i] for r in rows)[len(rows) // 2], max(r[i] for r in rows))
                       for i, nm in ((1, "loads"), (2, "first"), (3, "last"), (4, "end"))))
    rt = (C.c_ulonglong * 8)()
    lib.ewal_dbg_fr_result_steps(rt, 8)
    print("  fr_result thread 0 (cycles from its start): metadata %d, fence+sync %d, frames+ordinal %d, "
          "compose %d, host writes %d" % tuple(rt[i] - rt[0] for i in range(1, 6)))
    wt = (C.c_ulonglong * (8192 * 4))()
    lib.ewal_dbg_fr_wave_times(wt, 8192 * 4)
    ws = [(wt[w * 4], wt[w * 4 + 1], wt[w * 4 + 2]) for w in range(8192) if wt[w * 4 + 1]]
    if ws:   # s_memrealtime ticks at 100 MHz: 10 ns
        t0 = min(x[0] for x in ws)
        ends = sorted((x[1] - t0) / 100.0 for x in ws)
        starts = sorted((x[0] - t0) / 100.0 for x in ws)
        q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]   # noqa: E731
        tl = sorted(x[2] for x in ws)
        print("  wave start us: p50 %.1f p99 %.1f max %.1f | end us: p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f"
              " | tiles per wave p10 %d p50 %d p90 %d max %d" %
              (q(starts, .5), q(starts, .99), starts[-1], q(ends, .1), q(ends, .5), q(ends, .9), q(ends, .99),
               ends[-1], q(tl, .1), q(tl, .5), q(tl, .9), tl[-1]))
    waves = [list(t[w * 8:(w + 1) * 8]) for w in range(8192) if any(t[w * 8:(w + 1) * 8])]
    tot = [sum(x) for x in waves]
    print("%s: %d frames, %.3f GiB, device %.3f ms (stream %.3f), %d waves" %
          (label, n, nb / (1 << 30), rs.device_ms, rs.stream_ms, len(waves)))
    print("  per-wave total cycles: avg %.0f max %.0f" % (sum(tot) / len(tot), max(tot)))
    for i, nm in enumerate(NAMES):
        col = [x[i] for x in waves]
        print("  %-9s avg %10.0f  max %10.0f  share %5.1f%%" % (nm, sum(col) / len(col), max(col),
                                                             100.0 * sum(col) / max(1, sum(tot))))
    d.free()
    ctx.close()


which = sys.argv[1:] or ["wal", "c1"]
if "wal" in which:
    one("configs[1]", 8 << 30, 64, 65536)
if "c1" in which:
    one("configs[0]", int(285e6), 256, 256)
if "shards" in which:
    one("configs[2] x128 shards", 64 << 20, 128, 4096, nsh=128)
