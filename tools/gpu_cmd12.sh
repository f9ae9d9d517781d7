# A/B (wal + shards) plus per-kernel rocprof stats of both builds on configs[1]
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in A B; do
  EWAL_LIB_PATH=ablibs/libewal_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$L -o run -- python3 bench.py --workload wal --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prof_$L.log 2>&1
done
bash tools/gpu_ab.sh ${1:-3}
