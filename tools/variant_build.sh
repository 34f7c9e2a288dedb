#!/bin/bash
# Builds find-tfbs_amd/lib/probe<NAME>/libtfbs_amd.so with one source compiled under
# extra defines (timing variants; run with TFBS_LIB=find-tfbs_amd/lib/probe<NAME>/libtfbs_amd.so).
# Usage: tools/variant_build.sh SOURCE NAME:DEFINES[:FILE]...   (SOURCE: e.g. bgzf_gpu; FILE: another
# copy of that source, e.g. an older revision, compiled instead of find-tfbs_amd/csrc/SOURCE.hip)
set -e
cd "$(dirname "$0")/.."
make -s -j8 find-tfbs_amd/lib/libtfbs_amd.so
src=$1; shift
for spec in "$@"; do
  IFS=: read -r name extra file <<< "$spec"
  [ -z "$file" ] && file=find-tfbs_amd/csrc/$src.hip
  d=find-tfbs_amd/lib/probe$name
  mkdir -p $d
  flags=""
  [ "$src" = scan_mfma ] && flags="-mllvm -amdgpu-mfma-vgpr-form -ffinite-math-only"  # as the Makefile
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter --offload-arch=gfx950 -munsafe-fp-atomics \
    $flags -Ifind-tfbs_amd/csrc $extra -x hip -c $file -o $d/$src.o
  objs=$(ls find-tfbs_amd/lib/obj/*.o | grep -v "/$src.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libtfbs_amd.so $objs $d/$src.o -lz -lpthread
done
