# A/B: D = batched k_fc with contiguous tile runs + register-folded shard reductions; E = D + whole-line slot stores in k_stream; GPU suite on E
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_D.so ablibs/libewal_E.so" 3 "wal shards" > gpurun_out/ab25.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_E.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu25.txt 2>&1
