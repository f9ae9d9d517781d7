#!/bin/bash
# A/B of k_frame's resident workgroups per CU (EWAL_FRAME_WG) on one box.
cd /root/repo
mkdir -p gpurun_out
for wg in 3 4 2 3 4; do
  for w in wal shards; do
    EWAL_FRAME_WG=$wg timeout -k 10 120 python3 bench.py --workload $w --shards-per-gpu 128 --steps 20 --warmup 2 \
      --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w wg=$wg', d['value'], d['ms_per_step'], d.get('pipeline_device_ms'))" || exit 1
  done
done
