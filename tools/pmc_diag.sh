#!/bin/bash
# Diagnostic PMC passes for k_stream stalls (run ON the GPU box from the repo root).
set -e
out=${1:-gpurun_out/pmcd}; shift || true
export TMPDIR=/tmp
mkdir -p "$out"
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex k_stream --output-format csv -d "$out/$name" -o pmc -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --size-gib 4 > "$out/$name.log" 2>&1
}
run d1 SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_IFETCH SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_VMEM
run d2 SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT
run d3 TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run d4 TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES
run d5 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_IFETCH_LEVEL SQ_LEVEL_WAVES
