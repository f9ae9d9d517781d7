#!/bin/bash
# Builds etcd_amd/libewal.so for gfx950 (hipcc cross-compiles without a GPU).
set -euo pipefail
cd "$(dirname "$0")"
ARCH=${EWAL_ARCH:-gfx950}
hipcc --offload-arch=$ARCH -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result \
  -I../include -o libewal.so csrc/ewal_api.hip csrc/ewal_host.cpp csrc/ewal_join.cpp "$@"
