"""Timing of the GPU batched encoder (ewal_encode_entries_device) on N
entries of S bytes each (device-resident payload, one call timed by HIP-
synchronised wall clock after a warmup)."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
from etcd_amd import wal as W, _lib as L
from etcd_amd._lib import lib, check
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
size = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
ctx = W.Context(0)
payload = os.urandom(n * size)
arr = (L.EntryDesc * n)()
for i in range(n):
    arr[i].term, arr[i].index, arr[i].data_off, arr[i].data_len, arr[i].type = 7, i + 1, i * size, size, 0
cap = len(payload) + 80 * n + 64
dd, de, do = ctx.alloc(len(payload) + 64), ctx.alloc(C.sizeof(arr)), ctx.alloc(cap)
dd.upload(payload)
de.upload(bytes(arr))
out_len, crc = C.c_uint64(), C.c_uint32()
ts = []
for it in range(4):
    t = time.perf_counter()
    check(lib.ewal_encode_entries_device(ctx.handle, dd.ptr, len(payload), de.ptr, n, 0, do.ptr, cap,
                                         C.byref(out_len), C.byref(crc)))
    ts.append(time.perf_counter() - t)
t = sorted(ts[1:])[1]
print("entries %d x %d B: %.1f MB frames in %.3f ms -> %.1f GB/s (payload), crc %08x" %
      (n, size, out_len.value / 1e6, t * 1e3, len(payload) / t / 1e9, crc.value))
