#!/bin/bash
# rocprofv3 kernel trace + stats of one bench.py workload; summary to stdout.
# Usage: tools/prof_kernels.sh OUTDIR WORKLOAD [extra bench args]
cd /root/repo
OUT=$1; W=$2; shift 2
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --workload $W --steps 5 --warmup 1 \
  --no-cpu-baseline --no-e2e "$@" > $OUT.bench.json 2> $OUT.err || exit 1
python3 tools/prof_summary.py $OUT
