"""Host-side cost of one ReadAll call: the wall time of the C call (ctypes,
perf_counter) against the device pipeline's HIP-event time, per environment
variant of ONE library build (hooks builds: EWAL_SPIN, EWAL_NO_MID_EVENTS).
Usage: python3 tools/host_gap.py MODE ROUNDS LIB 'K=V+K=V' ...   MODE: wal | c1"""
import os
import subprocess
import sys

mode, rounds, lib, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
child = r'''
import ctypes as C, os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from etcd_amd import wal as W, _lib as L
mode = sys.argv[1]
ctx = W.Context(0)
size, lo, hi = (8 << 30, 64, 65536) if mode == "wal" else (285_000_000, 256, 256)
blob, n = W.synth_wal(size, lo, hi, seed=2)
d = ctx.alloc(len(blob) + 64)
d.upload_ptr(C.addressof((C.c_char * len(blob)).from_buffer(blob)), len(blob))
f = L.lib.ewal_readall_device
r = L.Result()
walls, devs = [], []
for i in range(22):
    t0 = time.perf_counter()
    f(ctx.handle, d.ptr, len(blob), 1, C.byref(r))
    t1 = time.perf_counter()
    assert r.status == 0
    if i >= 2:
        walls.append((t1 - t0) * 1e3); devs.append(r.device_ms)
walls.sort(); devs.sort()
t0 = time.perf_counter()
for i in range(20):
    f(ctx.handle, d.ptr, len(blob), 1, C.byref(r))
loop = (time.perf_counter() - t0) * 1e3 / 20
print("%.4f %.4f %.4f" % (walls[len(walls) // 2], devs[len(devs) // 2], loop))
'''
res = {v: [] for v in variants}
for rd in range(rounds):
    for v in variants:
        env = dict(os.environ, EWAL_LIB_PATH=os.path.abspath(lib))
        for kv in v.split("+"):
            k, _, val = kv.partition("=")
            if k != "X":
                env[k] = val
        out = subprocess.run([sys.executable, "-c", child, mode], env=env, capture_output=True, text=True, timeout=300)
        lines = [x for x in out.stdout.splitlines() if x.strip()]
        if out.returncode != 0 or not lines:
            print("round %d %s FAILED: %s" % (rd, v, out.stderr[-800:]), flush=True)
            sys.exit(1)
        w, dv, lp = map(float, lines[-1].split())
        res[v].append((w, dv, lp))
        print("round %d %-32s %s call wall %.4f ms  device %.4f ms  loop %.4f ms/call" % (rd, v, mode, w, dv, lp),
              flush=True)
for v in variants:
    m = lambda i: sorted(x[i] for x in res[v])[len(res[v]) // 2]   # noqa: E731
    print("%-32s %s median call wall %.4f device %.4f host %.4f loop %.4f" % (v, mode, m(0), m(1), m(0) - m(1), m(2)),
          flush=True)
