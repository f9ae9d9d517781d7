#!/bin/bash
# A/B of one library under environment settings, alternating (bench.py).
# Usage: tools/ab_env.sh "ENV_A" "ENV_B" [rounds] [workloads]
cd /root/repo
A=$1; B=$2; R=${3:-2}; WS=${4:-"wal shards"}
for r in $(seq $R); do
  for e in "$A" "$B"; do
    for w in $WS; do
      env $e timeout -k 10 150 python3 bench.py --workload $w --shards-per-gpu 128 --steps 10 --warmup 2 \
        --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e $w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)" || exit 1
    done
  done
done
