#!/bin/bash
# Builds variants of libcfd_amd.so that differ only in compile-time knobs of
# one Jacobi translation unit (VARIANT_TU, default cfd_jacobi_pipe2; e.g.
# cfd_jacobi_lds8, the kind-5 T = 8 launch), for A/B runs on the GPU:
#   CFD_LIB=cfd-demo_amd/lib/variants/<name>/libcfd_amd.so python tools/tb_one.py
# Usage: [VARIANT_TU=cfd_jacobi_lds8] tools/build_variants.sh name:"-DFLAG=1 -DOTHER=2" ...
set -e
cd "$(dirname "$0")/../cfd-demo_amd"
make -s -j8
TU=${VARIANT_TU:-cfd_jacobi_pipe2}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt"
case "$TU" in cfd_jacobi_lds*) FLAGS="$FLAGS -fno-slp-vectorize";; esac
OTHERS=$(ls build/*.o | grep -vF "/$TU.o")
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  mkdir -p lib/variants/$name
  /opt/rocm/bin/hipcc $FLAGS $defs -c csrc/$TU.hip -o lib/variants/$name/tu.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/variants/$name/libcfd_amd.so $OTHERS \
    lib/variants/$name/tu.o -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
  rm lib/variants/$name/tu.o
done
