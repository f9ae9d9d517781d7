"""Timing-only ablation of the frame pass (EWAL_STREAM_ABLATE bits 256: no
Record walk, 512: no Entry walk, 1024: no prefix_at): prints the device time
of the whole ReadAll and the rocprof-free split via HIP events is not
available per kernel, so run under rocprofv3 --stats for per-kernel times."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
from etcd_amd import wal as W
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
buf, n = W.synth_wal(int(gib * (1 << 30)), 64, 65536, seed=2)
ctx = W.Context(0)
d = ctx.alloc(len(buf) + 64)
d.upload_ptr(C.addressof((C.c_char * len(buf)).from_buffer(buf)), len(buf))
ms = []
for i in range(6):
    r = W.readall_device(d, len(buf), 1)
    ms.append(r.device_ms - r.stream_ms)
ms = sorted(ms[1:])
print("ablate=%s post-stream device ms median %.4f status %d" % (os.environ.get("EWAL_STREAM_ABLATE", "0"),
                                                             ms[len(ms) // 2], r.status))
