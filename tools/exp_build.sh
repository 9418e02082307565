#!/bin/bash
# Development: build experiment variants of the library, one per -DPG_EXP_BITS
# value, as pangenome_amd/libpangenome_hip_e<n>.so (load one with
# PG_LIB_NAME=libpangenome_hip_e<n>.so).  Never the product build.
set -eu
cd "$(dirname "$0")/../pangenome_amd/csrc"
for n in "$@"; do
  d=build_e$n; mkdir -p $d
  for f in pg_stage pg_parse pg_dbg pg_walk pg_persist pg_abi; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DPG_EXP_BITS=$n -c -o $d/$f.o $f.hip &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libpangenome_hip_e$n.so $d/*.o
done
