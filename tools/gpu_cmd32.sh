# A/B: L = k_uapply loads a dense unit's whole slot line up front, vs J (HEAD); configs[0] (c1) and configs[1]; GPU suite on L
set -e
mkdir -p gpurun_out
bash tools/ab_quick.sh "ablibs/libewal_J.so ablibs/libewal_L.so" 3 "c1 wal" > gpurun_out/ab32.log 2>&1
EWAL_LIB_PATH=ablibs/libewal_L.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu32.txt 2>&1
