# A/B: N1 = k_fc's seed shift by ternary digits (two bank-disjoint tables per digit, <= 11 steps), vs N0 (HEAD); GPU suite on N1
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_N0.so ablibs/libewal_N1.so" 3 "wal shards" > gpurun_out/ab34.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_N1.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu34.txt 2>&1
