#!/bin/bash
# HBM traffic of one kernel at a bench configuration (run ON the GPU box from
# the repo root): two PMC passes of their own (FETCH_SIZE, WRITE_SIZE; the
# gfx950 TCC slot limit keeps them apart), then tools/traffic.py turns them
# into profiles/<kernel>_pmc.json (per launch).
# Usage: tools/traffic.sh OUT [KERNEL_REGEX [bench.py args...]]
#   default: k_stream at the default bench line (configs[1])
set -e
out=${1:-gpurun_out/traffic}
kern=${2:-k_stream}
shift $(( $# > 2 ? 2 : $# ))
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 3 --warmup 1 --no-cpu-baseline --no-e2e)
export TMPDIR=/tmp
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c --kernel-include-regex "$kern" --output-format csv -d "$out/$c" -o pmc -- \
    python3 bench.py "${args[@]}" > "$out/$c.log" 2>&1
done
