#!/bin/bash
# Build A/B variants of libnydusgpu.so that differ only in blake3.hip compile
# flags, into nydus-snapshotter_amd/build/ab/NAME.so (run here, on the CPU).
# usage: scripts/build_ab.sh NAME "-DFLAG=V ..." [NAME "-D..."] ...
set -eu
cd "$(dirname "$0")/../nydus-snapshotter_amd"
make -s libnydusgpu.so
mkdir -p build/ab
OTHER=$(ls build/*.o | grep -v blake3.o)
while [ $# -ge 2 ]; do
  NAME=$1; FLAGS=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc $FLAGS \
    -c csrc/blake3.hip -o build/ab/blake3_$NAME.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/$NAME.so \
    build/ab/blake3_$NAME.o $OTHER -lcrypto -lz -ldl -lpthread
  echo "built build/ab/$NAME.so ($FLAGS)"
done
