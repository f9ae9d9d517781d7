#!/bin/bash
# Round-5 session 22: PMC traffic of the last build -- k_frames at configs[1],
# configs[0] and configs[2] (the spill reduction), k_stream at configs[1].
set -eo pipefail
out=${1:-gpurun_out/s22}
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/traffic.sh "$out/tr_wal" k_frames --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --configs none
python3 tools/traffic.py "$out/tr_wal" k_frames "configs[1] (bench.py default, 8 GiB)" wal
cp profiles/k_frames_pmc_wal.json "$out/"
bash tools/traffic.sh "$out/tr_c1" k_frames --workload c1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
python3 tools/traffic.py "$out/tr_c1" k_frames "configs[0] on the GPU (bench.py --workload c1, 286 MB)" c1
cp profiles/k_frames_pmc_c1.json "$out/"
bash tools/traffic.sh "$out/tr_shards" k_frames --workload shards --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
python3 tools/traffic.py "$out/tr_shards" k_frames "configs[2] (bench.py --workload shards: 512 x 64 MiB, 29.3 M frames)" shards
cp profiles/k_frames_pmc_shards.json "$out/"
bash tools/traffic.sh "$out/tr_stream" k_stream --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --configs none
python3 tools/traffic.py "$out/tr_stream" k_stream "configs[1] (bench.py default, 8 GiB)"
cp profiles/k_stream_pmc.json "$out/"
echo done
