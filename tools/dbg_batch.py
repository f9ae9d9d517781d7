"""Debug: the torn-shard batch of test_gpu_batch with EWAL_DEBUG output."""
import os
import random
import sys

os.environ["EWAL_DEBUG"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from etcd_amd import wal as W, _lib as L  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_parity import build_wal  # noqa: E402

ctx = W.Context(0)
rng = random.Random(11)
base = [build_wal(rng, 30, 500, big_terms=False) for _ in range(6)]
for name, shards in (("clean", base), ("torn", base[:2] + [base[2][:-5]] + base[3:])):
    res = W.readall_batch_bytes(shards, [0] * 6, ctx)
    print(name, [(r.status, r.flags, r.n_records, r.fail_record, r.fail_offset) for r in res], flush=True)
    print("oracle", [(O.readall(s, 0)["status"], O.readall(s, 0)["n_records"]) for s in shards], flush=True)
    print("lens", [len(s) for s in shards], "offs", [sum(len(x) for x in shards[:i]) for i in range(7)])
s5 = base[5]
g = W.readall_bytes(s5, 0, ctx)
print("single s5", g.status, g.n_records, g.fail_record)
offs = O.chain_crcs(s5)[1]
print("s5 frame offsets", offs)
for sh in range(6):   # each shard alone in a batch, and shard 5 with each predecessor
    r = W.readall_batch_bytes([base[sh]], [0], ctx)[0]
    print("alone", sh, r.status, r.n_records)
for k in range(5):
    r = W.readall_batch_bytes(base[k:], [0] * (6 - k), ctx)
    print("from", k, [(x.status, x.fail_record) for x in r])
