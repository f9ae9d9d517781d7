"""One process: an 8 GiB configs[1]-shaped WAL in HBM, 4 ReadAll calls (the
hooks library's EWAL_OV / EWAL_OV_NOFR select the pipeline) -- the target of
rocprofv3 --kernel-trace in tools/gpu_overlap.sh."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.getcwd())
import torch  # noqa: F401,E402
from etcd_amd import wal as W, _lib as L  # noqa: E402
ctx = W.Context(0)
buf, n = W.synth_wal(8 << 30, 64, 65536, seed=2)
d = ctx.alloc(len(buf) + 64)
d.upload_ptr(C.addressof((C.c_char * len(buf)).from_buffer(buf)), len(buf))
for i in range(4):
    r = L.Result()
    L.lib.ewal_readall_device(ctx.handle, d.ptr, len(buf), 1, C.byref(r))
    assert r.status == 0 and r.n_records == n, (r.status, r.n_records)
    print("call %d stream %.4f device %.4f post %.4f frames %.4f" % (i, r.stream_ms, r.device_ms, r.post_ms,
                                                                     r.frames_ms), flush=True)
