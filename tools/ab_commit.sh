#!/bin/bash
# A/B of two library builds on the configs[4] (maybeCommit) workload.
cd /root/repo
for r in 1 2; do for lib in "$1" "$2"; do
  EWAL_LIB_PATH=$lib timeout -k 10 120 python3 bench.py --workload commit --steps 50 --no-cpu-baseline 2>/dev/null | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib)', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1
done; done
