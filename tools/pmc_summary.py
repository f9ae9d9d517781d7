"""Summarise tools/pmc_stream.sh output: per-kernel mean of every counter
(one value per dispatch, summed over the per-XCD / per-SE instances that
rocprofv3 reports).  Usage: python3 tools/pmc_summary.py gpurun_out/pmc [kernel-substring]"""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
want = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for (d, cn), v in per.items():
        vals[names[d]][cn].append(v)
for k, cs in vals.items():
    if want and want not in k:
        continue
    print(k[:70])
    for cn in sorted(cs):
        v = cs[cn]
        print("   %-24s %16.1f  (n=%d)" % (cn, sum(v) / len(v), len(v)))
