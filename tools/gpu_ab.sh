#!/bin/bash
# One A/B call: tools/gpu_ab.sh NAME "MODE:ROUNDS ..." LIB...  -> gpurun_out/NAME/ab_MODE.txt
# (MODE: wal | shards | c1, tools/ab_run.py; each step under its own time limit)
set -o pipefail
NAME=$1; MODES=$2; shift 2
OUT=gpurun_out/$NAME
mkdir -p $OUT
for mr in $MODES; do
  m=${mr%%:*}; r=${mr##*:}
  timeout -k 10 400 python -u tools/ab_run.py $m $r "$@" > $OUT/ab_$m.txt 2>&1
  rc=$?; echo "rc=$rc: ab $m $r" >> $OUT/steps.txt
  grep median $OUT/ab_$m.txt
  [ $rc -eq 0 ] || exit $rc
done
