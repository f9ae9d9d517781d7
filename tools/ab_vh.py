"""A/B of the frame pass's 128-B prefixes (vh[]) inside ONE process on one
GPU (box-to-box spread is larger than the effect): two ctxs over the same
device-resident input, one with EWAL_OPT_VH_ON, one with EWAL_OPT_VH_OFF,
calls alternated; medians of device_ms / stream_ms / frames_ms.
Usage: python3 tools/ab_vh.py MODE ROUNDS   MODE: shards (configs[2]: 512 x
64 MiB per GPU, 128-4096 B entries) | wal (configs[1]) | c1 (configs[0])"""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: F401,E402
from etcd_amd import wal as W, _lib as L  # noqa: E402

mode, rounds = sys.argv[1], int(sys.argv[2])
nsh = int(os.environ.get("AB_SHARDS", "512"))
if mode == "shards":
    blob, lens, nrec = W.synth_shards(list(range(nsh)), 64 << 20, 128, 4096)
else:
    size, lo, hi = (8 << 30, 64, 65536) if mode == "wal" else (285_000_000, 256, 256)
    blob, n = W.synth_wal(size, lo, hi, seed=2)
    lens = [len(blob)]
print("input %.2f GiB, %d shard(s)" % (len(blob) / (1 << 30), len(lens)), flush=True)
ctxs = {"vh_on": W.Context(0), "vh_off": W.Context(0)}
ctxs["vh_on"].set_options(vh=True)
ctxs["vh_off"].set_options(vh=False)
d = ctxs["vh_on"].alloc(len(blob) + 64)
d.upload_ptr(C.addressof((C.c_char * len(blob)).from_buffer(blob)), len(blob))
del blob
ns = len(lens)
cl, cr = (C.c_uint64 * ns)(*lens), (C.c_uint64 * ns)(*([1] * ns))
times = {k: [] for k in ctxs}
verdict = {}


def call(ctx):
    if mode == "shards":
        co = (L.Result * ns)()
        assert L.lib.ewal_readall_batch_device(ctx.handle, d.ptr, ns, cl, cr, co) == 0
        assert all(x.status == 0 and not (x.flags & L.FLAG_SHARD_FALLBACK) for x in co)
        return co[0], tuple((x.status, x.n_records, x.last_crc) for x in co)
    r = L.Result()
    L.lib.ewal_readall_device(ctx.handle, d.ptr, lens[0], 1, C.byref(r))
    assert r.status == 0
    return r, (r.status, r.n_records, r.last_crc)


for rd in range(rounds):
    for k, ctx in ctxs.items():
        for i in range(4):
            r, v = call(ctx)
            verdict.setdefault(k, v)
            assert verdict[k] == v
            if i >= 1:
                times[k].append((r.device_ms, r.stream_ms, r.frames_ms))
    print("round %d done" % rd, flush=True)
assert verdict["vh_on"] == verdict["vh_off"], "results differ"
for k, t in times.items():
    dv, sv, fv = (statistics.median(x[j] for x in t) for j in range(3))
    print("%-7s %s device %.4f ms  stream %.4f ms  frames %.4f ms  (n=%d)" % (k, mode, dv, sv, fv, len(t)))
