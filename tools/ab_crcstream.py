"""A/B timing of k_stream<false> (ewal_crc32_update_device over 8 GiB of
random device bytes) between library builds in ONE GPU session; timing-only
ablation builds (EW_XS) return wrong CRCs.
Usage: python3 tools/ab_crcstream.py LIB... [--rounds R]"""
import os, subprocess, sys
libs = [a for a in sys.argv[1:] if a.endswith(".so")]
rounds = 2
child = r'''
import ctypes as C, os, sys
sys.path.insert(0, os.getcwd())
import torch
from etcd_amd import wal as W, _lib as L
lib = L.lib
lib.ewal_last_stream_ms.restype = C.c_float
lib.ewal_last_stream_ms.argtypes = [C.c_void_p]
n = 8 << 30
t = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
ctx = W.Context(0)
out = C.c_uint32()
ms = []
for i in range(10):
    rc = lib.ewal_crc32_update_device(ctx.handle, 0, L.CASTAGNOLI, C.c_void_p(t.data_ptr()), n, C.byref(out))
    assert rc == 0, rc
    if i >= 2:
        ms.append(lib.ewal_last_stream_ms(ctx.handle))
ms.sort()
print("%.4f" % ms[len(ms) // 2])
'''
res = {l: [] for l in libs}
for rd in range(rounds):
    for l in libs:
        env = dict(os.environ, EWAL_LIB_PATH=os.path.abspath(l))
        o = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=300)
        if o.returncode:
            print(o.stderr[-2000:])
            sys.exit(1)
        v = float(o.stdout.split()[-1])
        res[l].append(v)
        print("round %d %-20s k_stream<false> %.4f ms  %.1f GB/s" % (rd, os.path.basename(l), v, (8 << 30) / v / 1e6),
              flush=True)
