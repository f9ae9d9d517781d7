# instruction-cache counters for k_stream (wal = k_stream<true> sparse, shards = dense, snap = k_stream<false>) and k_fc
set -e
export TMPDIR=/tmp
out=gpurun_out/pmc_icache; mkdir -p $out
for w in wal shards snap; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS \
    --output-format csv -d $out/$w -o pmc -- python3 bench.py --workload $w --shards-per-gpu 128 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $out/$w.log 2>&1
done
