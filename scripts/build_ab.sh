#!/bin/bash
# Build A/B variants of libnydusgpu.so that differ only in one source's
# compile flags (AB_SRC, default blake3; AB_SRC=dedup with -DNGPU_PROBE_AB=1
# for the dict-probe variants), into nydus-snapshotter_amd/build/ab/NAME.so
# (run here, on the CPU).
# usage: [AB_SRC=dedup] scripts/build_ab.sh NAME "-DFLAG=V ..." [NAME "-D..."] ...
set -eu
cd "$(dirname "$0")/../nydus-snapshotter_amd"
make -s libnydusgpu.so
mkdir -p build/ab
SRC=${AB_SRC:-blake3}
OTHER=$(ls build/*.o | grep -v "/$SRC.o")
while [ $# -ge 2 ]; do
  NAME=$1; FLAGS=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc $FLAGS \
    -c csrc/$SRC.hip -o build/ab/${SRC}_$NAME.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/$NAME.so \
    build/ab/${SRC}_$NAME.o $OTHER -lcrypto -lz -ldl -lpthread
  echo "built build/ab/$NAME.so ($FLAGS)"
done
