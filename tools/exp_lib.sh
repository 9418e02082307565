#!/bin/bash
# Development: one experiment build of the library with extra compiler flags,
# as pangenome_amd/libpangenome_hip_<name>.so (load it with
# PG_LIB_NAME=libpangenome_hip_<name>.so).  Never the product build.
#   tools/exp_lib.sh <name> "<flags>" [git-rev]   (git-rev: build that revision's sources)
set -eu
name=$1; flags=$2; rev=${3:-}
root="$(cd "$(dirname "$0")/.." && pwd)"
src="$root/pangenome_amd/csrc"
d="$src/build_e_$name"; rm -rf "$d"; mkdir -p "$d"
if [ -n "$rev" ]; then                 # (the revision's tree, laid out as in the repository)
  t="$d/tree"; mkdir -p "$t/pangenome_amd/csrc" "$t/include"
  for f in $(git -C "$root" ls-tree --name-only "$rev" pangenome_amd/csrc/ | grep -E '\.(hip|h)$'); do
    git -C "$root" show "$rev:$f" > "$t/$f"
  done
  git -C "$root" show "$rev:include/pangenome.h" > "$t/include/pangenome.h"
  s="$t/pangenome_amd/csrc"
else
  s="$src"
fi
for f in pg_stage pg_parse pg_dbg pg_walk pg_persist pg_abi; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags -c -o "$d/$f.o" "$s/$f.hip" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$root/pangenome_amd/libpangenome_hip_$name.so" "$d"/*.o
echo "built libpangenome_hip_$name.so"
