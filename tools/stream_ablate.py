"""Timing-only ablation of k_stream (EWAL_STREAM_ABLATE set by the caller):
runs ReadAll on a synthetic WAL and prints the k_stream time.  Results of an
ablated run are meaningless (the CRC or the candidates are skipped)."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
from etcd_amd import wal as W
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
buf, n = W.synth_wal(int(gib * (1 << 30)), 64, 65536, seed=2)
ctx = W.Context(0)
d = ctx.alloc(len(buf) + 64)
d.upload_ptr(C.addressof((C.c_char * len(buf)).from_buffer(buf)), len(buf))
ms = []
for i in range(8):
    r = W.readall_device(d, len(buf), 1)
    ms.append(r.stream_ms)
ms = sorted(ms[2:])
print("ablate=%s R=%s k_stream ms median %.4f min %.4f -> %.1f GB/s  status %d" % (
    os.environ.get("EWAL_STREAM_ABLATE", "0"), os.environ.get("EWAL_STREAM_R", "16"), ms[len(ms) // 2], ms[0],
    len(buf) / ms[0] / 1e6, r.status))
