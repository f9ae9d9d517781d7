"""Kernel timeline of the last ReadAll calls from a rocprofv3 --kernel-trace
directory: per call (a k_stream launch starting at unit 0 opens a call) the
kernels in start order with start / end relative to the call's first kernel
(us).  Usage: python3 tools/ov_timeline.py TRACE_DIR [calls]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48],
                     r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Queue_Id", r.get("Stream_Id", ""))))
rows.sort()
# calls: split where a gap of > 200 us between kernel ends and the next start
calls, cur, last_end = [], [], None
for r in rows:
    if last_end is not None and r[0] - last_end > 200_000:
        calls.append(cur)
        cur = []
    cur.append(r)
    last_end = max(last_end or 0, r[1])
calls.append(cur)
for c in calls[-ncalls:]:
    t0 = c[0][0]
    print("---- call: %d kernels, %.1f us" % (len(c), (max(x[1] for x in c) - t0) / 1e3))
    for s, e, name, grid, q in c:
        print("  %9.1f %9.1f %8.1f  q=%-4s grid=%-8s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, grid, name))
