#!/bin/bash
# Builds etcd_amd/libewal.so for gfx950 (hipcc cross-compiles without a GPU)
# and libewal_synth.so, the synthetic-WAL generator of bench.py and the tests
# (host C++ only; not part of the product library).
set -euo pipefail
cd "$(dirname "$0")"
ARCH=${EWAL_ARCH:-gfx950}
hipcc --offload-arch=$ARCH -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result \
  -I../include -o libewal.so csrc/ewal_api.hip csrc/ewal_host.cpp csrc/ewal_join.cpp "$@"
g++ -O3 -std=c++17 -fPIC -shared -Wall -I../include -o libewal_synth.so csrc/ewal_synth.cpp \
  -L. -lewal -Wl,-rpath,'$ORIGIN' -lpthread
