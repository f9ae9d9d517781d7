#!/bin/bash
# PMC passes over the post-stream kernels of the bench (run ON the GPU box).
set -e
out=${1:-gpurun_out/pmcp}; shift || true
export TMPDIR=/tmp
mkdir -p "$out"
R='k_verify|k_decode|k_uagg|k_uapply|k_link|k_gap|k_ents|k_meta|k_tscan'
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex "$R" --output-format csv -d "$out/$name" -o pmc -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --size-gib 4 > "$out/$name.log" 2>&1
}
run f FETCH_SIZE
run w WRITE_SIZE
run s SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES
