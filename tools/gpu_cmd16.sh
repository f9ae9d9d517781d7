# k_stream<false> ablations (no CRC / no v stores) and wal without v stores, one box
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ab_crcstream.py ablibs/libewal_A.so ablibs/libewal_C.so ablibs/libewal_F.so ablibs/libewal_G.so > gpurun_out/ab16.log 2>&1
AB_NOCHECK=1 timeout -k 10 400 python3 tools/ab_stream.py ablibs/libewal_A.so ablibs/libewal_F.so 2 8 >> gpurun_out/ab16.log 2>&1
