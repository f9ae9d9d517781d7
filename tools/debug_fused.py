"""Fused vs general path vs oracle on random WALs (debug aid, GPU)."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O  # noqa: E402
from etcd_amd import wal as W  # noqa: E402
from test_gpu_parity import build_wal  # noqa: E402

os.environ["EWAL_FUSED"] = "0"
c0 = W.Context(0)
os.environ["EWAL_FUSED"] = "1"
c1 = W.Context(0)
bad = 0
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    rng = random.Random(seed)
    w = build_wal(rng, rng.randrange(1, 400), rng.choice([100, 3000, 70000]), cuts=rng.randrange(0, 3))
    if seed % 3 == 1:
        w = bytearray(w)
        w[rng.randrange(len(w))] ^= 1 << rng.randrange(8)
        w = bytes(w)
    for ri in (0, 1):
        o = O.readall(w, ri)
        g0 = W.readall_bytes(w, ri, c0).as_dict()
        g1 = W.readall_bytes(w, ri, c1).as_dict()
        keys = ("status", "fail_record", "fail_offset", "n_records", "last_crc", "enti", "metadata", "state")
        d0 = [k for k in keys if g0[k] != o[k] and not (k in ("last_crc", "enti", "metadata", "state") and o["status"])]
        d1 = [k for k in keys if g1[k] != o[k] and not (k in ("last_crc", "enti", "metadata", "state") and o["status"])]
        e1 = o["status"] == 0 and g1["ents"] != o["ents"]
        if d0 or d1 or e1:
            bad += 1
            print("seed", seed, "ri", ri, "len", len(w), "oracle", o["status"], o["fail_record"], o["n_records"],
                  "| general", d0, g0["status"], g0["fail_record"], "| fused", d1, e1, g1["status"], g1["fail_record"],
                  g1["n_records"], flush=True)
            if bad > 8:
                sys.exit(1)
print("mismatches", bad)
