import random, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_gpu_parity import build_wal
from test_gpu_fuzz import _mutate
from etcd_amd import wal as W
from oracle import oracle as O
ctx = W.Context(0)
for block in (1, 2, 3, 4):
    rng = random.Random(9100 + block)
    for it in range(6):
        shards, ris = [], []
        for _ in range(rng.randrange(2, 12)):
            w = build_wal(rng, rng.randrange(3, 60), rng.choice([40, 600, 3000]), cuts=rng.randrange(0, 2), big_terms=False)
            shards.append(_mutate(rng, w) if rng.random() < 0.5 else w)
            ris.append(rng.choice([0, 1, 5]))
        res = W.readall_batch_bytes(shards, ris, ctx)
        for s, (b, ri, r) in enumerate(zip(shards, ris, res)):
            o = O.readall(b, ri)
            if r.status != o["status"]:
                print("block", block, "it", it, "shard", s, "status", r.status, o["status"], "flags", r.flags, flush=True)
                continue
            if o["status"] == O.OK:
                g = [(x.Index, x.Term, x.Data) for x in r.ents]
                w = [(x["index"], x["term"], x["data"]) for x in o["ents"]]
                if g != w:
                    bad = [i for i in range(min(len(g), len(w))) if g[i] != w[i]]
                    print("block", block, "it", it, "shard", s, "of", len(shards), "ri", ri, "flags", hex(r.flags), "len", len(g), len(w),
                          "nbad", len(bad), "first", bad[:5], "gpu", g[bad[0]][:2] if bad else None,
                          "lens", [len(x) for x in shards], flush=True)
