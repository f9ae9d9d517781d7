set -e
mkdir -p gpurun_out
bash tools/gpu_ab.sh 3 "wal shards snap"
