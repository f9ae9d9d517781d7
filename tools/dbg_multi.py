"""Debug: the multi-ctx join of one fuzz case against the oracle (run ON the
GPU box).  Usage: python3 tools/dbg_multi.py SEED N"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O          # noqa: E402
from etcd_amd import wal as W          # noqa: E402
from test_gpu_fuzz import _large_case  # noqa: E402
from test_gpu_parity import gpu_readall  # noqa: E402


def diff(tag, got, want):
    d = [i for i in range(min(len(got), len(want))) if got[i] != want[i]]
    print(tag, "len", len(got), len(want), "ndiff", len(d), "first", d[:5], "last", d[-3:], flush=True)
    for i in d[:3]:
        print("   ", i, got[i], want[i])


seed, n = int(sys.argv[1]), int(sys.argv[2])
m, ri = _large_case(seed)
o = O.readall(m, ri)
want = [(e["index"], e["term"], e["data"][:8] if e["data"] else e["data"]) for e in o["ents"]]
ctxs = [W.Context(0) for _ in range(n)]
g = gpu_readall(ctxs[0], m, ri)
diff("single", [(e["index"], e["term"], e["data"][:8] if e["data"] else e["data"]) for e in g["ents"]], want)
mm = W.Multi(ctxs)
r = mm.readall(m, ri)
rows, starts = mm.rows()
print("starts", starts, "rows", [(x.status, x.deferred, x.n_records, x.ri) for x in rows], "resplit", mm.resplit)
diff("multi", [(e.Index, e.Term, e.Data[:8] if e.Data else e.Data) for e in r.ents], want)
st = list(starts) + [len(m)]
for k in range(n):
    part = m[st[k]:st[k + 1]]
    print("range", k, st[k], st[k + 1], flush=True)
    if k == 0:
        orr = O.readall(part, rows[k].ri)
        gr = gpu_readall(ctxs[0], part, rows[k].ri)
        print("  range0 alone: oracle", orr["status"], len(orr["ents"]), "gpu", gr["status"], len(gr["ents"]))
        if orr["status"] == O.OK:
            diff("  range0", [(e["index"], e["term"], e["data"][:8] if e["data"] else e["data"]) for e in gr["ents"]],
                 [(e["index"], e["term"], e["data"][:8] if e["data"] else e["data"]) for e in orr["ents"]])
