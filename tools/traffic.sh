#!/bin/bash
# HBM traffic of k_stream at the bench configuration (run ON the GPU box from
# the repo root): two PMC passes of their own (FETCH_SIZE, WRITE_SIZE; the
# gfx950 TCC slot limit keeps them apart), then tools/traffic.py turns them
# into profiles/k_stream_pmc.json (FETCH_SIZE x 2, the gfx950 correction of
# MI355X_MICROARCH.md "HBM", + WRITE_SIZE, per launch).
set -e
out=${1:-gpurun_out/traffic}
export TMPDIR=/tmp
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c --kernel-include-regex k_stream --output-format csv -d "$out/$c" -o pmc -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/$c.log" 2>&1
done
