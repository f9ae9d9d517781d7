"""profiles/<kernel>_pmc.json from tools/traffic.sh's two PMC passes:
per-launch HBM bytes = FETCH_SIZE (KiB) x 1024 x 2 (gfx950: FETCH_SIZE counts
half the bytes of a wide streaming read) + WRITE_SIZE (KiB) x 1024.
Usage: python3 tools/traffic.py ROOT [KERNEL [CONFIG [WORKLOAD]]]
  default: k_stream, configs[1] (bench.py default, 8 GiB); WORKLOAD names the
  file profiles/<kernel>_pmc_<workload>.json (bench.py reads it for that line).
Per counter, the median over the launches at least half as large as the
largest (the timed steps, not a ReadAll's one-frame warm-up call).  The x2
holds for the frame pass's 16-B-per-lane gathers too (calibrated:
profiles/r05/fetch_size_gather_calibration.txt, x2 = 1.09 x the distinct lines)."""
import csv, glob, json, os, re, sys
from collections import defaultdict
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_stream"
config = sys.argv[3] if len(sys.argv) > 3 else "configs[1] (bench.py default, 8 GiB)"
workload = sys.argv[4] if len(sys.argv) > 4 else None
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = defaultdict(float)
    for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            # the kernel itself, not others whose names contain it (k_frames_seam)
            if re.match(r"(void )?%s[<(]" % re.escape(kern), r["Kernel_Name"]) and r["Counter_Name"] == c:
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(per.values())
    v = [x for x in v if x >= v[-1] / 2] if v else v
    vals[c] = v[len(v) // 2] if v else None
fetch = vals["FETCH_SIZE"] * 1024 * 2
write = vals["WRITE_SIZE"] * 1024
out = {"kernel": kern, "config": config,
       "fetch_size_kib_median": vals["FETCH_SIZE"], "write_size_kib_median": vals["WRITE_SIZE"],
       "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
       "hbm_bytes_per_launch": fetch + write,
       "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts half of a wide streaming read; "
               "the same factor measured for 16-B-per-lane gathers, profiles/r05/fetch_size_gather_calibration.txt)"}
name = kern + "_pmc" + ("_" + workload if workload else "") + ".json"
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", name), "w"), indent=1)
print(json.dumps(out))
