#!/bin/bash
# Alternating A/B of library builds (bench.py, configs[1] and configs[2] at 128 shards).
# Usage: tools/ab_quick.sh "LIB_A LIB_B ..." [rounds] [workloads]
cd /root/repo
LIBS=$1; R=${2:-3}; WS=${3:-"wal shards"}
for r in $(seq $R); do
  for lib in $LIBS; do
    for w in $WS; do
      EWAL_LIB_PATH=$lib timeout -k 10 150 python3 bench.py --workload $w --shards-per-gpu 128 --steps 10 --warmup 2 \
        --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib) $w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)" || exit 1
    done
  done
done
