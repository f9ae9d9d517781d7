# k_stream ablations on one box: bare-read ceiling (membw), k_stream<false> (snap) with/without CRC and v stores, wal without v stores
set -e
mkdir -p gpurun_out
timeout -k 10 120 ./tools/membw 8 > gpurun_out/ab15.log 2>&1
bash tools/ab_quick.sh "ablibs/libewal_A.so ablibs/libewal_C.so ablibs/libewal_F.so ablibs/libewal_G.so" 2 "snap" >> gpurun_out/ab15.log 2>&1
AB_NOCHECK=1 timeout -k 10 400 python3 tools/ab_stream.py ablibs/libewal_A.so ablibs/libewal_F.so 2 8 >> gpurun_out/ab15.log 2>&1
