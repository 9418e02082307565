#!/bin/bash
# Development: libpangenome_hip_dbg.so, the library with PG_DEBUG_BOUNDS index
# checks (load it with PG_LIB_NAME=libpangenome_hip_dbg.so).  Never the product build.
set -eu
cd "$(dirname "$0")/../pangenome_amd/csrc"
d=build_dbg; mkdir -p $d
for f in pg_stage pg_parse pg_dbg pg_walk pg_persist pg_abi; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DPG_DEBUG_BOUNDS -c -o $d/$f.o $f.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libpangenome_hip_dbg.so $d/*.o
