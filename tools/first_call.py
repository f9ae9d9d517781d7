"""Where a fresh context's first ReadAll spends its time (diagnostic):
ctx create, hipMalloc of the workspace sizes, first ReadAll on a fresh ctx
(code objects not loaded yet), then a second fresh ctx in the same process."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from etcd_amd import wal as W, _lib as L  # noqa: E402

buf, n = W.synth_wal(int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 8 << 30, 64, 65536, seed=2)
nb = len(buf)
t = time.perf_counter(); ctx0 = W.Context(0); print("ctx_create ms", round((time.perf_counter() - t) * 1e3, 3))
d = ctx0.alloc(nb + 64)
d.upload_ptr(C.addressof((C.c_char * nb).from_buffer(buf)), nb)
for mb in (64, 512, 1024, 2048):
    p = C.c_void_p()
    t = time.perf_counter()
    L.lib.ewal_device_alloc(ctx0.handle, mb << 20, C.byref(p))
    dt = time.perf_counter() - t
    L.lib.ewal_device_free(ctx0.handle, p)
    print("hipMalloc %d MiB ms" % mb, round(dt * 1e3, 3))
for name in ("first ctx, first call", "first ctx, 2nd call"):
    t = time.perf_counter(); r = W.readall_device(d, nb, 1); dt = time.perf_counter() - t
    print(name, "ms", round(dt * 1e3, 3), "device_ms", round(r.device_ms, 3), r.status)
for i in range(2):
    c2 = W.Context(0)
    if i == 1 and hasattr(L.lib, "ewal_ctx_reserve"):
        t = time.perf_counter(); L.lib.ewal_ctx_reserve(c2.handle, nb, 0); print("reserve ms", round((time.perf_counter() - t) * 1e3, 3))
    r = L.Result()
    t = time.perf_counter(); L.lib.ewal_readall_device(c2.handle, d.ptr, nb, 1, C.byref(r)); dt = time.perf_counter() - t
    print("fresh ctx%s, first call ms" % (" (reserved)" if i else ""), round(dt * 1e3, 3), "device_ms", round(r.device_ms, 3))
    t = time.perf_counter(); L.lib.ewal_readall_device(c2.handle, d.ptr, nb, 1, C.byref(r)); dt = time.perf_counter() - t
    print("  2nd call ms", round(dt * 1e3, 3))
    c2.close()
