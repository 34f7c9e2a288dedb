#!/bin/bash
# Builds find-tfbs_amd/lib/probe<N>/libtfbs_amd.so with scan_mfma.hip compiled
# under -DTFBS_MFMA_PROBE=N (bottleneck probes; see scan_mfma.hip).  Run with
# TFBS_LIB=find-tfbs_amd/lib/probe<N>/libtfbs_amd.so python tools/tune.py ...
set -e
cd "$(dirname "$0")/.."
make -s -j8 find-tfbs_amd/lib/libtfbs_amd.so
# Each argument: N, or NAME:N:DEFINES (e.g. w1:0:-DTFBS_MFMA_DEEP_WT=1 builds
# lib/probew1 with probe 0 and the extra define).
for spec in "$@"; do
  IFS=: read -r name n extra <<< "$spec"
  [ -z "$n" ] && n=$name
  d=find-tfbs_amd/lib/probe$name
  mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form -ffinite-math-only \
    -DTFBS_MFMA_PROBE=$n $extra -x hip -c find-tfbs_amd/csrc/scan_mfma.hip -o $d/scan_mfma.o
  objs=$(ls find-tfbs_amd/lib/obj/*.o | grep -v scan_mfma.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libtfbs_amd.so $objs $d/scan_mfma.o -lz -lpthread
done
