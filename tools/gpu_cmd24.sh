# A/B: ents store deferred behind the next tile's loads (C) vs HEAD (A); then the GPU suite on C
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_C.so" 3 "wal shards" > gpurun_out/ab24.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu24.txt 2>&1
