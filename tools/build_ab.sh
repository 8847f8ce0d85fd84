#!/bin/bash
# A/B library: tigerbeetle_amd/libtbc_<tag>.so built from the working tree with
# extra compiler flags (e.g. -DNAME=VALUE); bench.py / tests pick it with
# TBC_LIB=tigerbeetle_amd/libtbc_<tag>.so. usage: build_ab.sh TAG FLAGS...
set -e
TAG=${1:?tag}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/tbc_ab_$TAG; mkdir -p $B
cd $ROOT/tigerbeetle_amd/csrc
for f in aegis merge sort kway grid engine; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -Wno-unused-value \
    -Wno-unused-result -I../../include "$@" -c $f.hip -o $B/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $B/*.o -o $ROOT/tigerbeetle_amd/libtbc_$TAG.so
echo built tigerbeetle_amd/libtbc_$TAG.so
