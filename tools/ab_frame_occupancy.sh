#!/bin/bash
cd /root/repo
for r in 1 2; do
  for cfg in "etcd_amd/libewal.so 3" "abtmp/libewal_w4.so 3" "abtmp/libewal_w4.so 4"; do
    set -- $cfg
    for w in wal shards; do
      EWAL_LIB_PATH=$1 EWAL_FRAME_WG=$2 timeout -k 10 150 python3 bench.py --workload $w --shards-per-gpu 128 --steps 10 --warmup 2 \
        --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $1) wg$2 $w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('pipeline_device_ms'))" || exit 1
    done
  done
done
