#!/bin/bash
# Round-5 probes (run ON the GPU box from the repo root): how k_stream's and
# k_frames' times scale with the CUs they get (hooks build, grid caps), and
# the SQ counters of k_frames on configs[1] and on 128 configs[2] shards.
set -eo pipefail
out=${1:-gpurun_out/probe}
mkdir -p "$out"
export TMPDIR=/tmp
L=ablibs/libewal_hooks.so
timeout -k 10 400 python3 -u tools/env_sweep.py wal 2 $L "X=0" EWAL_STREAM_CUS=224 EWAL_STREAM_CUS=192 \
  EWAL_STREAM_CUS=160 EWAL_STREAM_CUS=128 EWAL_FRAME_CUS=128 EWAL_FRAME_CUS=64 > "$out/sweep_wal.txt" 2>&1
AB_SHARDS=128 timeout -k 10 300 python3 -u tools/env_sweep.py shards 2 $L "X=0" EWAL_STREAM_CUS=192 \
  EWAL_STREAM_CUS=128 EWAL_FRAME_CUS=128 > "$out/sweep_shards.txt" 2>&1
pmc() {  # name workload-args... -- counters
  local name=$1; shift
  local args=()
  while [ "$1" != "--" ]; do args+=("$1"); shift; done
  shift
  timeout -k 10 150 rocprofv3 --pmc "$@" --kernel-include-regex "k_frames|k_stream" --output-format csv \
    -d "$out/$name" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --configs none \
    "${args[@]}" > "$out/$name.log" 2>&1
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR"
pmc wal_sq1 --workload wal -- $SQ1
pmc wal_sq2 --workload wal -- $SQ2 GRBM_GUI_ACTIVE
pmc sh_sq1 --workload shards --shards-per-gpu 128 -- $SQ1
pmc sh_sq2 --workload shards --shards-per-gpu 128 -- $SQ2 GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py "$out" > "$out/pmc_summary.txt" 2>&1 || true
echo done
