#!/bin/bash
# Development: build experiment variants of the library, one per -DPG_EXP_BITS
# value, as pangenome_amd/libpangenome_hip_e<n>.so (load one with
# PG_LIB_NAME=libpangenome_hip_e<n>.so).  Never the product build.  Only
# pg_dbg.hip reads PG_EXP_BITS: the other objects are built once, in
# build_e_common.
set -eu
cd "$(dirname "$0")/../pangenome_amd/csrc"
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics"
mkdir -p build_e_common
for f in pg_stage pg_parse pg_walk pg_persist pg_abi; do
  [ build_e_common/$f.o -nt $f.hip ] && [ build_e_common/$f.o -nt pg_internal.h ] || $HIPCC -c -o build_e_common/$f.o $f.hip &
done
wait
for n in "$@"; do
  d=build_e$n; mkdir -p $d
  $HIPCC -DPG_EXP_BITS=$n -c -o $d/pg_dbg.o pg_dbg.hip &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libpangenome_hip_e$n.so build_e$n/pg_dbg.o build_e_common/*.o
done
