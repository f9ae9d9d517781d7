"""Diagnostics of the frame pass on the bench workload: per call, the device
time, candidates, chain runs and frames left to the general walker."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
from etcd_amd import wal as W
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
buf, n = W.synth_wal(int(gib * (1 << 30)), 64, 65536, seed=2)
ctx = W.Context(0)
d = ctx.alloc(len(buf) + 64)
d.upload_ptr(C.addressof((C.c_char * len(buf)).from_buffer(buf)), len(buf))
for i in range(4):
    r = W.readall_device(d, len(buf), 1)
    print("call %d status %d n %d cand %d runs %d slow %d device_ms %.4f stream_ms %.4f" %
          (i, r.status, r.n_records, r.n_candidates, r.n_runs, r.n_slow, r.device_ms, r.stream_ms))
