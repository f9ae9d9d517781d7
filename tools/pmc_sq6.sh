#!/bin/bash
# Round 6: the SQ counter passes (issue / wait / LDS) of the final build's
# k_frames and k_stream, configs[2]-shaped shards (128 x 64 MiB) and configs[1]
# (run ON the GPU box from the repo root; then tools/pmc_summary.py OUT).
set -eo pipefail
out=${1:-gpurun_out/pmc6}
export TMPDIR=/tmp
mkdir -p "$out"
run() {  # name workload-args -- counters...
  local name=$1; shift
  local args=()
  while [ "$1" != "--" ]; do args+=("$1"); shift; done
  shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o pmc -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e "${args[@]}" > "$out/$name.log" 2>&1
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
run wal_sq1 --configs none -- $SQ1
run wal_sq2 --configs none -- $SQ2
run shards_sq1 --workload shards --shards-per-gpu 128 -- $SQ1
run shards_sq2 --workload shards --shards-per-gpu 128 -- $SQ2
echo done
