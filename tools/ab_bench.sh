#!/bin/bash
# A/B of two library builds on one box through bench.py workloads.
# Usage: tools/ab_bench.sh LIB_A LIB_B [rounds]
cd /root/repo
A=$1; B=$2; R=${3:-2}
for r in $(seq $R); do
  for lib in $A $B; do
    for w in wal c1 shards; do
      EWAL_LIB_PATH=$lib timeout -k 10 150 python3 bench.py --workload $w --shards-per-gpu 128 --steps 10 --warmup 2 \
        --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib) $w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1
    done
  done
done
