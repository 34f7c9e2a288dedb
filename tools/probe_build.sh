#!/bin/bash
# Builds find-tfbs_amd/lib/probe<N>/libtfbs_amd.so with scan_mfma.hip compiled
# under -DTFBS_MFMA_PROBE=N (bottleneck probes; see scan_mfma.hip).  Run with
# TFBS_LIB=find-tfbs_amd/lib/probe<N>/libtfbs_amd.so python tools/tune.py ...
set -e
cd "$(dirname "$0")/.."
make -s -j8 find-tfbs_amd/lib/libtfbs_amd.so
for n in "$@"; do
  d=find-tfbs_amd/lib/probe$n
  mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form \
    -DTFBS_MFMA_PROBE=$n -x hip -c find-tfbs_amd/csrc/scan_mfma.hip -o $d/scan_mfma.o
  objs=$(ls find-tfbs_amd/lib/obj/*.o | grep -v scan_mfma.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libtfbs_amd.so $objs $d/scan_mfma.o -lz -lpthread
done
