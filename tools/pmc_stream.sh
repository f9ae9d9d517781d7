#!/bin/bash
# PMC passes over the bench's kernels (run ON the GPU box, from the repo root).
# Each pass is its own rocprofv3 run (gfx950 slot limits, MI355X_MICROARCH.md).
# Usage: tools/pmc_stream.sh OUTDIR [bench args]
set -e
out=${1:-gpurun_out/pmc}; shift || true
export TMPDIR=/tmp
mkdir -p "$out"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o pmc -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
}
BENCH_ARGS=("$@")
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
