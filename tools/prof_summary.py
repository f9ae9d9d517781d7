"""Per-kernel summary of a rocprofv3 --kernel-trace run: calls, average, and
the median of the calls at least half as long as the longest (the bench's
timed steps; a ReadAll's one-frame warm-up calls are left out), in us.
Usage: python3 tools/prof_summary.py OUTDIR   (the rocprofv3 -d directory)"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
per = defaultdict(list)
for r in csv.DictReader(open(f)):
    per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(per.items(), key=lambda kv: -sum(kv[1]))
for name, d in rows[:16]:
    mx = max(d)
    big = [x for x in d if x >= 0.5 * mx]
    print("%-60s calls %4d avg_us %9.1f median_big_us %9.1f" % (name[:60], len(d), sum(d) / len(d),
                                                                 statistics.median(big)))
