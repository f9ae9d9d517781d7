#!/bin/bash
# rocprofv3 kernel trace + stats of every bench workload the default line
# carries (run ON the GPU box from the repo root); summaries and the
# kernel_stats CSVs land in gpurun_out/prof_r04/ (copy to profiles/r04/).
set -e
out=gpurun_out/prof_r04
mkdir -p $out
for w in wal c1 shards snap commit rewind; do
  bash tools/prof_kernels.sh $out/$w $w --configs none > $out/$w.summary.txt
  cp "$(find $out/$w -name '*kernel_stats.csv' | head -1)" $out/${w}_kernel_stats.csv
done
