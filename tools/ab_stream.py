"""A/B timing of the ReadAll pipeline between library builds in ONE GPU
session (box-to-box variance is ~10%, larger than most single changes).
Usage: python3 tools/ab_stream.py LIB_A LIB_B [rounds] [gib]
Each round runs every library in its own process (the .so is chosen with
EWAL_LIB_PATH) and prints median k_stream and pipeline device times."""
import os, subprocess, sys
libs = sys.argv[1:3]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
gib = sys.argv[4] if len(sys.argv) > 4 else "8"
child = r'''
import ctypes as C, os, sys
sys.path.insert(0, os.getcwd())
import torch
from etcd_amd import wal as W
buf, n = W.synth_wal(int(float(sys.argv[1]) * (1 << 30)), 64, 65536, seed=2)
ctx = W.Context(0)
d = ctx.alloc(len(buf) + 64)
d.upload_ptr(C.addressof((C.c_char * len(buf)).from_buffer(buf)), len(buf))
s, p = [], []
for i in range(12):
    r = W.readall_device(d, len(buf), 1)
    assert r.status == 0 or os.environ.get('AB_NOCHECK')
    if i >= 2:
        s.append(r.stream_ms); p.append(r.device_ms)
s.sort(); p.sort()
print("%.4f %.4f" % (s[len(s) // 2], p[len(p) // 2]))
'''
res = {l: [] for l in libs}
for rd in range(rounds):
    for l in libs:
        env = dict(os.environ, EWAL_LIB_PATH=os.path.abspath(l))
        out = subprocess.run([sys.executable, "-c", child, gib], env=env, capture_output=True, text=True, timeout=300)
        line = [x for x in out.stdout.splitlines() if x.strip()][-1]
        sm, pm = map(float, line.split())
        res[l].append((sm, pm))
        print("round %d %-28s stream %.4f ms  pipeline %.4f ms" % (rd, os.path.basename(l), sm, pm), flush=True)
for l in libs:
    v = sorted(res[l])
    print("%-28s median stream %.4f pipeline %.4f" % (os.path.basename(l), v[len(v) // 2][0],
                                                     sorted(x[1] for x in v)[len(v) // 2]))
