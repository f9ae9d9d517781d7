# GPU suite on the radix-4 seed shift + per-shard fold in the seam, then A/B against HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu23.txt 2>&1
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_B.so" 3 "wal shards" > gpurun_out/ab23.log 2>&1
