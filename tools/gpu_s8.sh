#!/bin/bash
# Round-5 session 8: the split2 sub-line alone, k_frames PMC traffic at the
# configs[1] and configs[0] lines, a configs[0] frame-pass sweep (hooks build)
# and the kernel stats of every workload.  Run ON the GPU box from the repo root.
set -eo pipefail
out=${1:-gpurun_out/s8}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --configs split2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e \
  > "$out/bench_split2.json" 2> "$out/bench_split2.err"
bash tools/traffic.sh "$out/tr_wal" k_frames --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --configs none
python3 tools/traffic.py "$out/tr_wal" k_frames "configs[1] (bench.py default, 8 GiB)" wal
cp profiles/k_frames_pmc_wal.json "$out/"
bash tools/traffic.sh "$out/tr_c1" k_frames --workload c1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
python3 tools/traffic.py "$out/tr_c1" k_frames "configs[0] on the GPU (bench.py --workload c1, 286 MB)" c1
cp profiles/k_frames_pmc_c1.json "$out/"
timeout -k 10 600 python3 tools/env_sweep.py c1 2 ablibs/libewal_hooks.so X=0 EWAL_FRAME_CUS=128 \
  EWAL_FRAME_CUS=192 EWAL_FRAME_CUS=224 > "$out/sweep_c1.txt" 2>&1
p="$out/prof"
mkdir -p "$p"
for w in wal c1 shards snap commit rewind; do
  bash tools/prof_kernels.sh "$p/$w" $w --configs none > "$p/$w.summary.txt"
  cp "$(find "$p/$w" -name '*kernel_stats.csv' | head -1)" "$p/${w}_kernel_stats.csv"
done
echo done
