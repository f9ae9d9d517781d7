import os, random, struct, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_gpu_parity import build_wal
from etcd_amd import wal as W
from oracle import oracle as O
rng = random.Random(11)
base = [build_wal(rng, 30, 500, big_terms=False) for _ in range(6)]
ctx = W.Context(0)
b0 = bytes(base[0]) + struct.pack("<q", 3) + b"\x00\x01\x02"
print("single alone", flush=True)
g = W.readall_bytes(b0, 0, ctx) if hasattr(W, "readall_bytes") else None
print("single", g and (g.status, g.fail_record), O.readall(b0, 0)["status"], flush=True)
t3 = [b0] + [bytes(x) for x in base[1:]]
res = W.readall_batch_bytes(t3, [0] * 6, ctx)
print("batch", [(r.status, r.fail_record, r.flags) for r in res], flush=True)
