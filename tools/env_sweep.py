"""Timing of ONE library build under environment variants in one GPU session
(hooks builds: EWAL_STREAM_CUS / EWAL_FRAME_CUS / EWAL_TSH ...).
Usage: python3 tools/env_sweep.py MODE ROUNDS LIB 'K=V+K=V' ...   MODE: wal | shards | c1
Each round runs every library in its own process (EWAL_LIB_PATH) and prints
the median k_stream and pipeline device times of 10 calls (after 2 warmups);
AB_NOCHECK=1 skips the verdict check (timing-only ablation builds)."""
import os
import subprocess
import sys

mode, rounds, lib, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
child = r'''
import ctypes as C, os, sys
sys.path.insert(0, os.getcwd())
import torch
from etcd_amd import wal as W, _lib as L
mode = sys.argv[1]
ctx = W.Context(0)
if mode == "shards":
    nsh = int(os.environ.get("AB_SHARDS", "128"))
    blob, lens, nrec = W.synth_shards(list(range(nsh)), 64 << 20, 128, 4096)
else:
    size, lo, hi = (8 << 30, 64, 65536) if mode == "wal" else (285_000_000, 256, 256)
    blob, n = W.synth_wal(size, lo, hi, seed=2)
    lens = [len(blob)]
d = ctx.alloc(len(blob) + 64)
d.upload_ptr(C.addressof((C.c_char * len(blob)).from_buffer(blob)), len(blob))
ns = len(lens)
cl, cr, co = (C.c_uint64 * ns)(*lens), (C.c_uint64 * ns)(*([1] * ns)), (L.Result * ns)()
s, p = [], []
for i in range(12):
    if mode == "shards":
        assert L.lib.ewal_readall_batch_device(ctx.handle, d.ptr, ns, cl, cr, co) == 0
        r = co[0]
        ok = all(x.status == 0 and not (x.flags & L.FLAG_SHARD_FALLBACK) for x in co)
    else:
        r = L.Result()
        L.lib.ewal_readall_device(ctx.handle, d.ptr, lens[0], 1, C.byref(r))
        ok = r.status == 0
    assert ok or os.environ.get("AB_NOCHECK"), "verdict"
    if i >= 2:
        s.append(r.stream_ms); p.append(r.device_ms)
s.sort(); p.sort()
print("%.4f %.4f" % (s[len(s) // 2], p[len(p) // 2]))
'''
res = {v: [] for v in variants}
for rd in range(rounds):
    for v in variants:
        env = dict(os.environ, EWAL_LIB_PATH=os.path.abspath(lib))
        for kv in filter(None, v.split("+")):
            k, x = kv.split("=")
            env[k] = x
        out = subprocess.run([sys.executable, "-c", child, mode], env=env, capture_output=True, text=True,
                             timeout=300)
        lines = [x for x in out.stdout.splitlines() if x.strip()]
        if out.returncode != 0 or not lines:
            print("round %d %s FAILED: %s" % (rd, v, out.stderr[-800:]), flush=True)
            sys.exit(1)
        sm, pm = map(float, lines[-1].split())
        res[v].append((sm, pm))
        print("round %d %-32s %s stream %.4f ms  pipeline %.4f ms" % (rd, v, mode, sm, pm), flush=True)
for v in variants:
    st = sorted(x[0] for x in res[v])
    pp = sorted(x[1] for x in res[v])
    print("%-32s %s median stream %.4f pipeline %.4f" % (v, mode, st[len(st) // 2], pp[len(pp) // 2]), flush=True)
