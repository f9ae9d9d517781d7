# PMC passes over k_fc (bench shards at 128 shards), one counter set per rocprofv3 run
set -e
export TMPDIR=/tmp
out=gpurun_out/pmc_fc; mkdir -p $out
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$n -o pmc -- python3 bench.py --workload shards --shards-per-gpu 128 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $out/$n.log 2>&1; }
run ta TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
run sq SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
