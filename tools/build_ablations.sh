#!/bin/bash
# Diagnostic builds: each removes one cost from the trace kernels (images are wrong; timing only).
set -e
cd "$(dirname "$0")/../python-raytracer_amd/csrc"
OUT=${ABL_OUT:-../../build/abl}; mkdir -p $OUT
for f in ${ABL:-SHADOW POW TEX FB APPEND QSTORE NOSHADE PROF}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -munsafe-fp-atomics \
    -DRT_ABL_$f $( [ $f = PROF ] && echo -DRT_PROF ) -o $OUT/libsightpy_hip_$f.so rt_kernels.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
wait
ls -la $OUT
